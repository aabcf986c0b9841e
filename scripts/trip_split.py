#!/usr/bin/env python3
"""Where one traversal trip's time goes.

For each config (depth-1 configs: c2, c3), one frame through rt_wave_timeline after a few
warm-up frames (so the adaptive longest-first block order is the product's), then:
  * per wave: closest-hit main-loop trips and time (t_trace - t_pro_end), and with a library
    built with -DRTK_TL_SPLIT=1 the trips' memory wait (ticks from issuing a trip's record
    loads to all four having arrived) -> ns per trip = wait + the rest (VALU/SALU/LDS);
  * the frame's critical wave (ends last) and its longest wave, and the heavy waves (>= 64 trips);
  * the same block ALONE on the chip: a 16x16 window of the frame at the same pixel density
    (image-plane vectors scaled, so the rays are as coherent as in the frame; double-rounding
    makes them not bit-identical) rendered as a one-block frame, warmed, then stamped: what the
    critical wave's trips cost with the chip to itself.
Usage: RTAMD_LIB=... python3 scripts/trip_split.py OUT.json [c2 c3]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))
TICK_NS = 10.0   # s_memrealtime: 100 MHz


def wave_stats(rec, i):
    main = int(rec["main_c"][i])
    dur = float(rec["t_trace"][i] - rec["t_pro_end"][i]) * TICK_NS
    out = {"main_trips": main, "prologue_trips": int(rec["pro_c"][i]), "main_loop_ns": round(dur, 1),
           "ns_per_main_trip": round(dur / main, 1) if main else None,
           "wave_us": round(float(rec["t1"][i] - rec["t0"][i]) * TICK_NS / 1e3, 2),
           "start_us": round(float(rec["t0"][i] - rec["t0"].min()) * TICK_NS / 1e3, 2)}
    if "wait_c" in rec and main:
        wait = float(rec["wait_c"][i]) * TICK_NS
        out.update({"wait_ns_per_trip": round(wait / main, 1), "rest_ns_per_trip": round((dur - wait) / main, 1),
                    "trips_waiting_250ns_or_more": int(rec["longwait_c"][i])})
    return out


def group_stats(rec, mask):
    m = rec["main_c"][mask].astype(np.float64)
    dur = (rec["t_trace"][mask] - rec["t_pro_end"][mask]).astype(np.float64) * TICK_NS
    ok = m > 0
    out = {"waves": int(ok.sum()), "ns_per_main_trip": round(float(dur[ok].sum() / m[ok].sum()), 1) if ok.any() else None}
    if "wait_c" in rec and ok.any():
        wait = rec["wait_c"][mask].astype(np.float64)[ok] * TICK_NS
        out.update({"wait_ns_per_trip": round(float(wait.sum() / m[ok].sum()), 1),
                    "rest_ns_per_trip": round(float((dur[ok].sum() - wait.sum()) / m[ok].sum()), 1),
                    "share_of_trips_waiting_250ns_or_more": round(float(rec["longwait_c"][mask][ok].sum() / m[ok].sum()), 3)})
    return out


def window_params(p, W, H, x0, y0, n=16):
    """Params of an n x n window at (x0, y0) of a W x H frame at the frame's pixel density:
    image_pos = c + a xf + b yf with xf = (x - 0.5) / w (volumeRender.cl:1169-1190)."""
    q = p.copy().reshape(8, 4)
    a, b, c = q[0, :3].astype(np.float64), q[1, :3].astype(np.float64), q[2, :3].astype(np.float64)
    q[2, :3] = (c + a * (x0 / W) + b * (y0 / H)).astype(np.float32)
    q[0, :3] = (a * (n / W)).astype(np.float32)
    q[1, :3] = (b * (n / H)).astype(np.float32)
    return q.reshape(32)


def run(name):
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    r = rtamd.Renderer(0)
    r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    p = rtamd.params_to_array(mesh.camera_params(w, h))
    r.set_params(p)
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    lat = []
    for _ in range(30):
        t1 = time.perf_counter()
        r.render_device(w, h, depth, flags, dev.data_ptr())
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t1) * 1e3)
    tl = r.wave_timeline(w, h, depth, flags)
    rec = tl["launches"][0]
    crit = int(np.argmax(rec["t1"]))
    longest = int(np.argmax(rec["t1"] - rec["t0"]))
    res = {"config": name, "split": tl["split"], "frame_latency_ms_median": round(float(np.median(lat[5:])), 4),
           "timeline_frame_ms": tl["frame_ns"] / 1e6,
           "critical_wave": wave_stats(rec, crit), "longest_wave": wave_stats(rec, longest),
           "heavy_waves_64": group_stats(rec, rec["main_c"] >= 64),
           "all_waves": group_stats(rec, rec["main_c"] >= 1)}
    # the longest wave's block alone: a 16x16 window of the frame at the same pixel density
    tb = int(rec["tag"][longest])
    tiles_x = (w + 15) // 16
    x0, y0 = (tb % tiles_x) * 16, (tb // tiles_x) * 16
    wave_in_block = longest % 4
    r.set_params(window_params(p, w, h, x0, y0))
    small = torch.zeros(256, dtype=torch.int32, device="cuda")
    for _ in range(10):
        r.render_device(16, 16, depth, flags, small.data_ptr())
    torch.cuda.synchronize()
    alone = []
    for _ in range(5):
        t1 = r.wave_timeline(16, 16, depth, flags)["launches"][0]
        alone.append(wave_stats(t1, wave_in_block))
    res["longest_wave_block_alone"] = {"tile": tb, "x0": x0, "y0": y0, "wave": wave_in_block, "runs": alone}
    r.close()
    return res


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or ["c2", "c3"]
    res = {"library": os.environ.get("RTAMD_LIB", "product"), "configs": []}
    for n in names:
        x = run(n)
        print(json.dumps(x), flush=True)
        res["configs"].append(x)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
