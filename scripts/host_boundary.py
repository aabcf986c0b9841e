"""rt_render (the reference's own boundary: synchronous, frame read back into host memory,
raytrace_gpgpu at RayTracer.cpp:330-344) timed on a BASELINE config, into pinned and pageable
host memory; the frame is checked against one device-resident render (rt_render_device) of
the same camera.  Loads the library named by RTAMD_LIB (A/B of rt_render's row groups).
    python scripts/host_boundary.py [config] [frames]"""
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

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cfg = configs.CONFIGS[name]
w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
mesh, bvh, _ = configs.make_scene(cfg, threads=16)
r = rtamd.Renderer(0)
r.upload(rtamd.Scene.from_mesh(mesh, bvh))
r.set_params(rtamd.params_to_array(mesh.camera_params(w, h)))
dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
r.render_device(w, h, depth, flags, dev.data_ptr())
torch.cuda.synchronize()
want = dev.cpu().numpy().view(np.uint32)
res = {"config": name, "lib": rtamd.LIB_PATH, "digest": rtamd.library_digest()}
for kind in ("pinned", "pageable"):
    buf = torch.zeros(w * h, dtype=torch.int32, pin_memory=True) if kind == "pinned" else None
    arr = np.zeros(w * h, np.uint32)
    ptr = buf.data_ptr() if buf is not None else arr.ctypes.data
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:   # clock ramp
        r.render_host_ptr(w, h, depth, flags, ptr)
    t0 = time.perf_counter()
    for _ in range(n):
        r.render_host_ptr(w, h, depth, flags, ptr)
    ms = (time.perf_counter() - t0) / n * 1e3
    got = buf.numpy().view(np.uint32) if buf is not None else arr
    res[kind] = {"ms_per_frame": round(ms, 4), "equal_to_device_frame": bool(np.array_equal(got, want))}
print(json.dumps(res), flush=True)
