#!/usr/bin/env python3
"""Where a frame's time goes, wave by wave.

For each config: the BASELINE scene and camera, frames rendered one at a time on the ctx
stream (each synchronised: nothing overlaps the frame, as in bench.py's frame_latency), then
one frame through rt_wave_timeline (the stamping instantiation of the same kernels, with the
adaptive block order those frames built).  Per launch it reports:
  * span: first wave start -> last wave end (s_memrealtime, 100 MHz), against the frame's
    HIP-event time;
  * dispatch: how wave start times spread (a wave starts when a slot frees up);
  * the critical wave: the wave that ends last -- its start (late dispatch), its traversal
    trips (main loop + wave-uniform prologue) and time per trip;
  * epilogue: from the last wave's rays to the end of the launch (the in-kernel longest-first
    sort in the frame's last block);
  * per-XCD end times.
Plus rt_chase_latency: the dependent traversal-shaped iteration on 1 CU, on 1 wave per SIMD
and at 8 waves per SIMD (the latency roof's t_iter).
Usage: python3 scripts/wave_timeline.py OUTDIR [c2 c3 c5 ...] [--frames N]
Writes OUTDIR/timeline_<cfg>.json (+ .npz of the raw records)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def pct(a, q):
    return float(np.percentile(a, q)) if len(a) else 0.0


def summarize(rec, us_per_tick=0.01):
    t0, t1, t2 = rec["t0"], rec["t1"], rec["t2"]
    trips = rec["main"] + rec["prologue"]
    dur = (t1 - t0) * us_per_tick
    last = int(np.argmax(t1))
    longest = int(np.argmax(t1 - t0))
    work = trips > 0
    out = {
        "waves": int(len(t0)),
        "waves_with_traversal": int(work.sum()),
        "span_us": round(float(t2.max() - t0.min()) * us_per_tick, 2),
        "rays_end_us": round(float(t1.max() - t0.min()) * us_per_tick, 2),
        "epilogue_tail_us": round(float(t2.max() - t1.max()) * us_per_tick, 2),
        "start_us": {q: round(pct(t0 - t0.min(), q) * us_per_tick, 2) for q in (50, 90, 99, 100)},
        "wave_us": {q: round(pct(dur, q), 2) for q in (50, 90, 99, 100)},
        "wave_us_with_traversal": {q: round(pct(dur[work], q), 2) for q in (50, 90, 99, 100)},
        "trips": {q: round(pct(trips[work], q), 1) for q in (50, 90, 99, 100)},
        "trips_total": int(trips.sum()),
        "critical_wave": {"index": last, "start_us": round(float(t0[last] - t0.min()) * us_per_tick, 2),
                          "duration_us": round(float(dur[last]), 2), "trips_main": int(rec["main"][last]),
                          "trips_prologue": int(rec["prologue"][last]), "tag": int(rec["tag"][last]),
                          "xcc": int(rec["xcc"][last])},
        "longest_wave": {"index": longest, "start_us": round(float(t0[longest] - t0.min()) * us_per_tick, 2),
                         "duration_us": round(float(dur[longest]), 2), "trips_main": int(rec["main"][longest]),
                         "trips_prologue": int(rec["prologue"][longest])},
        "xcc_end_us": {int(x): round(float(t2[rec["xcc"] == x].max() - t0.min()) * us_per_tick, 2)
                       for x in np.unique(rec["xcc"])},
        "xcc_waves": {int(x): int((rec["xcc"] == x).sum()) for x in np.unique(rec["xcc"])},
    }
    # phases of a wave (first launch: its 64 rays; bounce launch: its last group): closest-hit
    # traversal, shading, shadow traversal; durations, and least-squares cost per trip of each
    # traversal (duration ~ a * main trips + b * prologue trips + c) over the waves of the launch
    if "t_trace" in rec and rec.get("bounce", 0) == 0:
        tt, ts = rec["t_trace"], rec["t_shade"]
        ok = work & (tt >= 0)
        sh = ok & (ts >= 0)
        te, tp = rec["t_enter"], rec["t_pro_end"]
        ph = {"setup_us": (te - t0)[ok] * us_per_tick, "prologue_us": (tp - te)[ok] * us_per_tick,
              "main_loop_us": (tt - tp)[ok] * us_per_tick,
              "closest_us": (tt - t0)[ok] * us_per_tick, "shade_us": (ts - tt)[sh] * us_per_tick,
              "shadow_us": (t1 - ts)[sh] * us_per_tick}
        out["phase_us"] = {k: {q: round(pct(v, q), 2) for q in (50, 90, 100)} for k, v in ph.items()}
        out["phase_us_total"] = {k: round(float(v.sum()), 1) for k, v in ph.items()}

        def fit(dur, m, p, mask):
            if mask.sum() < 16:
                return None
            A = np.stack([m[mask], p[mask], np.ones(mask.sum())], 1).astype(np.float64)
            coef = np.linalg.lstsq(A, dur[mask].astype(np.float64), rcond=None)[0]
            return {"ns_per_main_trip": round(float(coef[0]) * 1e3, 1), "ns_per_prologue_trip": round(float(coef[1]) * 1e3, 1),
                    "ns_fixed": round(float(coef[2]) * 1e3, 1)}
        out["fit_closest"] = fit((tt - t0) * us_per_tick, rec["main_c"], rec["pro_c"], ok)
        out["fit_shadow"] = fit((t1 - ts) * us_per_tick, rec["main_s"], rec["pro_s"], sh)
    if "main_c" in rec:
        out["trips_by_kind"] = {k: int(rec[k].sum()) for k in ("main_c", "pro_c", "main_s", "pro_s")}
    heavy = work & (trips >= 64)
    if heavy.any():
        per = dur[heavy] / trips[heavy] * 1e3
        out["ns_per_trip_heavy_waves"] = {q: round(pct(per, q), 1) for q in (10, 50, 90)}
    # busy wave-slots over time: how full the chip is as the launch drains
    edges = np.linspace(t0.min(), t2.max(), 21)
    live = [int(((t0 <= e) & (t2 > e)).sum()) for e in edges[:-1]]
    out["live_waves_at_5pct_steps"] = live
    return out


def run_config(name, outdir, frames):
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    scene = rtamd.Scene.from_mesh(mesh, bvh)
    p = mesh.camera_params(cfg["w"], cfg["h"])
    r = rtamd.Renderer(0)
    r.upload(scene)
    r.set_params(p)
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    lat, kern = [], []
    for _ in range(frames):
        t1 = time.perf_counter()
        r.render_device(w, h, depth, flags, dev.data_ptr())
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t1) * 1e3)
        kern.append(r.last_timing()[0])
    res = {"config": name, "frames_before": frames,
           "frame_latency_ms_median": round(float(np.median(lat[1:])), 4),
           "frame_kernels_ms_median": round(float(np.median(kern[1:])), 4)}
    tl = r.wave_timeline(w, h, depth, flags)
    res["timeline_frame_kernels_ms"] = tl["frame_ns"] / 1e6
    res["timeline_first_launch_ms"] = tl["first_ns"] / 1e6
    res["launches"] = [summarize(rec) for rec in tl["launches"]]
    np.savez_compressed(os.path.join(outdir, f"timeline_{name}.npz"),
                        **{f"l{k}_{f}": v for k, rec in enumerate(tl["launches"]) for f, v in rec.items()})
    # lone waves: the same scene and camera at 16x16 (one block: 4 waves on one CU) and 128x64
    # (32 blocks): per-trip time of the traversal when a wave has its CU (almost) to itself
    lone = {}
    for lw, lh in ((16, 16), (128, 64)):
        r.set_params(mesh.camera_params(lw, lh))
        for _ in range(5):
            r.render_device(lw, lh, depth, flags, dev.data_ptr())
        torch.cuda.synchronize()
        tl1 = r.wave_timeline(lw, lh, depth, flags)
        rec = tl1["launches"][0]
        trips = rec["main"] + rec["prologue"]
        dur = (rec["t1"] - rec["t0"]) * 10.0   # ns
        k = trips > 0
        lone[f"{lw}x{lh}"] = {"waves": int(len(trips)), "frame_us": tl1["frame_ns"] / 1e3,
                              "ns_per_trip": round(float(dur[k].sum() / trips[k].sum()), 1) if k.any() else None,
                              "max_trips": int(trips.max()), "max_wave_us": round(float(dur.max()) / 1e3, 2)}
    res["lone_waves"] = lone
    r.set_params(p)
    # four frames in flight, as bench.py times them
    res["inflight4"] = inflight(r, w, h, depth, flags, 4)
    # and the same frame with the static block order (RT_FLAG_STATIC_ORDER = 16)
    tls = r.wave_timeline(w, h, depth, flags | 16)
    res["static_order"] = {"frame_kernels_ms": tls["frame_ns"] / 1e6,
                           "first_launch": summarize(tls["launches"][0])}
    r.close()
    return res


def inflight_only(name, sizes):
    import torch
    import rtamd
    from rtamd import configs
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    r = rtamd.Renderer(0)
    r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    r.set_params(mesh.camera_params(cfg["w"], cfg["h"]))
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    for _ in range(5):
        r.render_device(w, h, depth, flags, dev.data_ptr())
    torch.cuda.synchronize()
    res = {"config": name}
    for k in sizes:
        res[f"inflight{k}"] = inflight(r, w, h, depth, flags, k)
    r.close()
    return res


def inflight(r, w, h, depth, flags, frames, slots=8192):
    """`frames` frames in flight (one stream each, rt_wave_timeline): how the launches of the
    frames share the chip over time -- live waves per launch kind in 20 steps of the span, the
    mean waves per SIMD over the span (wave-time / span / SIMDs), and each frame's span."""
    tl = r.wave_timeline(w, h, depth, flags, frames=frames)
    L = tl["launches"]
    t_lo = min(int(x["t0"].min()) for x in L)
    t_hi = max(int(x["t2"].max()) for x in L)
    edges = np.linspace(t_lo, t_hi, 21)
    kinds = sorted({x["bounce"] for x in L})
    live = {f"bounce{k}": [int(sum(((x["t0"] <= e) & (x["t2"] > e)).sum() for x in L if x["bounce"] == k))
                           for e in edges[:-1]] for k in kinds}
    wave_time = sum(float((x["t2"] - x["t0"]).sum()) for x in L)
    span = t_hi - t_lo
    frames_span = {}
    for f in range(frames):
        xs = [x for x in L if x["frame"] == f]
        frames_span[f] = round((max(int(x["t2"].max()) for x in xs) - min(int(x["t0"].min()) for x in xs)) / 100.0, 1)
    # the middle half of the span (frames overlapping, neither ramp nor drain of the burst)
    m_lo, m_hi = t_lo + 0.25 * span, t_lo + 0.75 * span
    mid_time = sum(float((np.minimum(x["t2"], m_hi) - np.maximum(x["t0"], m_lo)).clip(min=0).sum()) for x in L)
    return {"frames": frames, "span_us": round(span / 100.0, 1), "us_per_frame": round(span / 100.0 / frames, 1),
            "mean_waves_per_simd": round(wave_time / span / (slots / 8), 3),
            "mean_waves_per_simd_mid_half": round(mid_time / (0.5 * span) / (slots / 8), 3),
            "frame_span_us": frames_span, "live_waves_at_5pct_steps": live}


def chase(outdir):
    import torch
    import rtamd
    r = rtamd.Renderer(0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = {"cus": cus}
    for label, blocks in (("one_cu_4_waves", 1), ("1_wave_per_simd", cus), ("8_waves_per_simd", cus * 8)):
        for group in (4, 64):
            best = min(r.chase_latency(blocks, 16384, 512, group)[0] for _ in range(3))
            out[f"{label}_group{group}_ns_per_iter"] = round(best * 1e6 / 512, 1)
    r.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("configs", nargs="*", default=["c2", "c3", "c5"])
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--no-chase", action="store_true")
    ap.add_argument("--inflight-only", type=int, nargs="*", default=None,
                    help="only the frames-in-flight bursts, of these sizes (1..8)")
    a = ap.parse_args()
    os.makedirs(a.outdir, exist_ok=True)
    if a.inflight_only:
        for name in a.configs:
            res = inflight_only(name, a.inflight_only)
            with open(os.path.join(a.outdir, f"inflight_{name}.json"), "w") as f:
                json.dump(res, f, indent=1)
            print(json.dumps(res), flush=True)
        return
    if not a.no_chase:
        c = chase(a.outdir)
        print(json.dumps({"chase": c}), flush=True)
        with open(os.path.join(a.outdir, "chase_latency.json"), "w") as f:
            json.dump(c, f, indent=1)
    for name in a.configs:
        res = run_config(name, a.outdir, a.frames)
        with open(os.path.join(a.outdir, f"timeline_{name}.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
