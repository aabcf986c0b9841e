#!/usr/bin/env python3
"""A wave's phases from rt_wave_timeline (C3, C2): the wave-uniform prologue's trips against the
main loop's, start to traversal, shading, shadow ray + store; for the full frame and for the
block of the frame's longest wave alone (scripts/trip_split.py window_params).  Writes
gpurun_out/prologue.json.  C2 renders without shadow rays: its shade_us is not
stamped (negative)."""
import sys, os, json
sys.path.insert(0, "real-time-opencl-raytracer_amd"); sys.path.insert(0, "scripts")
import numpy as np, torch, rtamd
from rtamd import configs
from trip_split import window_params
out = {}
for name, (x0, y0) in (("c3", (1856, 704)), ("c2", (1232, 608))):
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    r = rtamd.Renderer(0); r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    p = rtamd.params_to_array(mesh.camera_params(w, h)); r.set_params(p)
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    for _ in range(10): r.render_device(w, h, depth, flags, dev.data_ptr())
    torch.cuda.synchronize()
    def stats(rec):
        pro_ns = (rec["t_pro_end"] - rec["t_enter"]).astype(np.float64) * 10
        main_ns = (rec["t_trace"] - rec["t_pro_end"]).astype(np.float64) * 10
        ok = (rec["pro_c"] > 0) & (rec["t_enter"] >= 0) & (rec["t_pro_end"] >= 0)
        okm = (rec["main_c"] > 0) & ok
        pre = (rec["t_enter"] - rec["t0"]).astype(np.float64) * 10
        shade = (rec["t_shade"] - rec["t_trace"]).astype(np.float64) * 10
        end = (rec["t1"] - rec["t_shade"]).astype(np.float64) * 10
        return {"pro_ns_per_trip": round(float(pro_ns[ok].sum() / rec["pro_c"][ok].sum()), 1),
                "main_ns_per_trip": round(float(main_ns[okm].sum() / rec["main_c"][okm].sum()), 1),
                "pro_trips_mean": round(float(rec["pro_c"][ok].mean()), 2), "main_trips_mean": round(float(rec["main_c"][ok].mean()), 2),
                "start_to_traversal_us": round(float(np.median(pre[ok])) / 1e3, 2),
                "shade_us": round(float(np.median(shade[ok])) / 1e3, 2), "shadow_and_store_us": round(float(np.median(end[ok])) / 1e3, 2),
                "wave_us_median": round(float(np.median((rec["t1"] - rec["t0"])[ok])) * 10 / 1e3, 2)}
    full = r.wave_timeline(w, h, depth, flags)["launches"][0]
    r.set_params(window_params(p, w, h, x0, y0))
    small = torch.zeros(256, dtype=torch.int32, device="cuda")
    for _ in range(10): r.render_device(16, 16, depth, flags, small.data_ptr())
    torch.cuda.synchronize()
    lone = r.wave_timeline(16, 16, depth, flags)["launches"][0]
    out[name] = {"full_frame": stats(full), "lone_block": stats(lone)}
    print(name, json.dumps(out[name]), flush=True)
    r.close()
json.dump(out, open("gpurun_out/prologue.json", "w"), indent=1)
