#!/usr/bin/env python3
"""One frame alone (bench.py's frame_latency: launch + device synchronize, host clock) split into
the host's enqueue (rt_render_device's own clock, rt_last_enqueue_time), the frame's kernels
(rt_last_timing: HIP events), and the rest (dispatch latency + the host noticing completion),
with three ways of waiting: torch.cuda.synchronize (bench.py's), the stream's synchronize, and
rt_render into pinned memory (the library's own spin-then-yield wait, wait_ctx).
Usage: python3 scripts/latency_split.py OUT.json [c2 c3]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def run(name, n=41):
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    r = rtamd.Renderer(0)
    r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    r.set_params(rtamd.params_to_array(mesh.camera_params(w, h)))
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    launch = r.frame_launcher(w, h, depth, flags)
    res = {"config": name}
    for how in ("device_sync", "stream_sync"):
        tot, enq, ker = [], [], []
        for i in range(n):
            t0 = time.perf_counter()
            launch(dev.data_ptr(), s.cuda_stream)
            t1 = time.perf_counter()
            if how == "device_sync":
                torch.cuda.synchronize()
            else:
                s.synchronize()
            t2 = time.perf_counter()
            if i:
                tot.append((t2 - t0) * 1e3)
                enq.append((t1 - t0) * 1e3)
                ker.append(r.last_timing()[0])
        res[how] = {"frame_ms_median": round(float(np.median(tot)), 4), "enqueue_ms_median": round(float(np.median(enq)), 4),
                    "kernels_ms_median": round(float(np.median(ker)), 4),
                    "rest_ms_median": round(float(np.median(np.array(tot) - np.array(enq) - np.array(ker))), 4)}
    pin = torch.zeros(w * h, dtype=torch.int32, pin_memory=True)
    tot, ker = [], []
    for i in range(n):
        t0 = time.perf_counter()
        r.render_host_ptr(w, h, depth, flags, pin.data_ptr())
        t2 = time.perf_counter()
        if i:
            tot.append((t2 - t0) * 1e3)
            ker.append(r.last_timing()[0])
    res["rt_render_pinned"] = {"frame_ms_median": round(float(np.median(tot)), 4), "kernels_ms_median": round(float(np.median(ker)), 4)}
    r.close()
    return res


def main():
    out = sys.argv[1]
    res = [run(c) for c in (sys.argv[2:] or ["c2", "c3"])]
    for x in res:
        print(json.dumps(x), flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
