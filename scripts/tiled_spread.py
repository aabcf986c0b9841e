#!/usr/bin/env python3
"""How far apart rt_render_tiled's contexts start their frame.

n contexts (default 8) on device 0 (the one-GPU box; each its own stream, as on n GPUs), the
scene uploaded once and copied (rt_scene_copy), frames rendered with rt_render_tiled into pinned
memory.  Per frame: the spread of the contexts' enqueue starts (rt_last_enqueue_time, host
steady clock), the last enqueue's end after the first start, and the frame's wall time; with
the per-context host threads (default) and with every part enqueued on the caller's thread
(RTAMD_TILED_WORKERS=0, the round-5 flow).
Usage: python3 scripts/tiled_spread.py OUT.json [config] [n] [frames]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def main():
    out = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "c3"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    rs = [rtamd.Renderer(0) for _ in range(n)]
    rs[0].upload(rtamd.Scene.from_mesh(mesh, bvh))
    for r in rs[1:]:
        r.copy_scene_from(rs[0])
    rs[0].set_params(mesh.camera_params(w, h))
    pinned = torch.zeros(w * h, dtype=torch.int32, pin_memory=True)
    ref = rs[0].render(w, h, depth, flags)
    res = {"config": name, "contexts": n, "device": 0, "frames": frames, "runs": {}}
    for mode in ("workers", "caller_thread"):
        os.environ["RTAMD_TILED_WORKERS"] = "1" if mode == "workers" else "0"
        spread, enq, wall = [], [], []
        for i in range(frames + 20):
            t0 = time.perf_counter_ns()
            rtamd.render_tiled(rs, w, h, depth, flags, out=pinned.data_ptr())
            t1 = time.perf_counter_ns()
            if i < 20:
                continue
            st = [r.last_enqueue_time() for r in rs]
            b = [x[0] for x in st]
            e = [x[1] for x in st]
            spread.append((max(b) - min(b)) / 1e3)
            enq.append((max(e) - min(b)) / 1e3)
            wall.append((t1 - t0) / 1e3)
        same = bool(np.array_equal(pinned.numpy().view(np.uint32), ref))
        q = lambda a, p: round(float(np.percentile(a, p)), 2)
        res["runs"][mode] = {"start_spread_us": {"p50": q(spread, 50), "p90": q(spread, 90), "max": q(spread, 100)},
                             "first_start_to_last_enqueue_end_us": {"p50": q(enq, 50), "p90": q(enq, 90)},
                             "frame_wall_us": {"p50": q(wall, 50), "p90": q(wall, 90)},
                             "frame_equals_rt_render": same}
        print(mode, json.dumps(res["runs"][mode]), flush=True)
    for r in rs:
        r.close()
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
