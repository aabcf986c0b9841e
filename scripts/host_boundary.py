"""rt_render (the reference's own boundary: synchronous, frame read back into host memory,
raytrace_gpgpu at RayTracer.cpp:330-344) timed on a BASELINE config, into pinned and pageable
host memory; the frame is checked against one device-resident render (rt_render_device) of
the same camera.  With --tiled N also rt_render_tiled over N contexts (device 0 repeated on a
one-GPU box: the N-GPU code path, not N GPUs' speed).  Loads the library named by RTAMD_LIB
(A/B); RTAMD_SYNC=block makes the library wait with hipStreamSynchronize instead of polling.
    python scripts/host_boundary.py [config] [frames] [--tiled N ...]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "real-time-opencl-raytracer_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config", nargs="?", default="c3")
ap.add_argument("frames", nargs="?", type=int, default=200)
ap.add_argument("--tiled", type=int, nargs="*", default=[])
ap.add_argument("--tiny", action="store_true",
                help="also rt_render of 8x8 and 64x64 frames (one block): the boundary's fixed cost")
a = ap.parse_args()
name, n = a.config, a.frames
cfg = configs.CONFIGS[name]
w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
mesh, bvh, _ = configs.make_scene(cfg, threads=16)
r = rtamd.Renderer(0)
r.upload(rtamd.Scene.from_mesh(mesh, bvh))
params = rtamd.params_to_array(mesh.camera_params(w, h))
r.set_params(params)
dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
r.render_device(w, h, depth, flags, dev.data_ptr())
torch.cuda.synchronize()
want = dev.cpu().numpy().view(np.uint32)
res = {"config": name, "lib": rtamd.LIB_PATH, "digest": rtamd.library_digest(),
       "sync": os.environ.get("RTAMD_SYNC", "query (default)")}


def timed(fn, ptr):
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:   # clock ramp
        fn(ptr)
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn(ptr)
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    return {"ms_per_frame": round(float(ts.mean()), 4), "ms_median": round(float(np.median(ts)), 4),
            "ms_p10": round(float(np.percentile(ts, 10)), 4)}


def run(label, fn):
    for kind in ("pinned", "pageable"):
        buf = torch.zeros(w * h, dtype=torch.int32, pin_memory=True) if kind == "pinned" else None
        arr = np.zeros(w * h, np.uint32)
        ptr = buf.data_ptr() if buf is not None else arr.ctypes.data
        out = timed(fn, ptr)
        got = buf.numpy().view(np.uint32) if buf is not None else arr
        out["equal_to_device_frame"] = bool(np.array_equal(got, want))
        res[f"{label}_{kind}"] = out


run("rt_render", lambda p: r.render_host_ptr(w, h, depth, flags, p))
if a.tiny:
    for tw, th in ((8, 8), (64, 64)):
        r.set_params(mesh.camera_params(tw, th))
        pin = torch.zeros(tw * th, dtype=torch.int32, pin_memory=True)
        res[f"rt_render_{tw}x{th}_pinned"] = timed(lambda p: r.render_host_ptr(tw, th, depth, flags, p), pin.data_ptr())
        d2 = torch.zeros(tw * th, dtype=torch.int32, device="cuda")
        def dev_sync(_p):
            r.render_device(tw, th, depth, flags, d2.data_ptr())
            torch.cuda.synchronize()
        res[f"render_device_sync_{tw}x{th}"] = timed(dev_sync, 0)
        res[f"kernels_{tw}x{th}_ms"] = round(r.last_timing()[0], 4)
    r.set_params(params)
for k in a.tiled:
    rs = [rtamd.Renderer(0) for _ in range(k)]
    rs[0].copy_scene_from(r)
    rs[0].set_params(params)
    for q in rs[1:]:
        q.copy_scene_from(r)
    run(f"tiled{k}", lambda p, rs=rs: rtamd.render_tiled(rs, w, h, depth, flags, out=p))
    for q in rs:
        q.close()
print(json.dumps(res), flush=True)
