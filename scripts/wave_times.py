"""Diagnostic: per-wave timeline of the fused render kernel (build variant `wt`,
-DRTK_WAVE_TIMES=1).  Renders the bench frame with RTAMD_WAVE_TIMES set, then
summarises how busy the chip is over the launch: resident waves over time, the
tail after the last wave starts, per-XCD finish times and per-wave durations.

    RTAMD_LIB=real-time-opencl-raytracer_amd/lib/variants/librtamd_wt.so \
        python scripts/wave_times.py [--config c3]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "real-time-opencl-raytracer_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wave_times.bin"))
    ap.add_argument("--shard", default="", help="R/N: one rank's bands of an N-way split (8-row bands)")
    args = ap.parse_args()
    import torch
    import bench
    import rtamd
    cfg = bench.CONFIGS[args.config]
    mesh, bvh, _ = bench.make_scene(cfg, 16)
    scene = rtamd.Scene.from_mesh(mesh, bvh)
    w, h = cfg["w"], cfg["h"]
    r = rtamd.Renderer(0)
    r.upload(scene)
    r.set_params(rtamd.params_to_array(mesh.camera_params(w, h)))
    tiling = None
    hl = h
    if args.shard:
        sr, sn = (int(v) for v in args.shard.split("/"))
        tiling = rtamd.rt_tiling(sr, sn, 8, 0)
        hl = rtamd.tiling_pixels(w, h, sr, sn, 8) // w
    out = torch.zeros(w * hl, dtype=torch.int32, device="cuda")
    for _ in range(3):
        r.render_device(w, h, cfg["depth"], cfg["flags"], out.data_ptr(), tiling=tiling)
    torch.cuda.synchronize()
    os.environ["RTAMD_WAVE_TIMES"] = args.out
    r.render_device(w, h, cfg["depth"], cfg["flags"], out.data_ptr(), tiling=tiling)
    torch.cuda.synchronize()
    print("kernel ms (with stamps):", r.last_kernel_ms())

    wt = np.fromfile(args.out, dtype=np.uint32).reshape(-1, 4)
    # pixel -> wave: 8x8 tiles (lane = pixel in the tile)
    px = np.arange(w * hl)
    x, y = px % w, px // w
    wave = (y // 8) * ((w + 7) // 8) + (x // 8)
    t0 = wt[:, 0].astype(np.int64)
    t1 = wt[:, 1].astype(np.int64)
    base = t0[t0 > 0].min()
    t0 -= base
    t1 -= base
    nw = wave.max() + 1
    ws = np.full(nw, np.iinfo(np.int64).max)
    we = np.zeros(nw, np.int64)
    np.minimum.at(ws, wave, t0)
    np.maximum.at(we, wave, t1)
    lane_busy = (t1 - t0).astype(np.float64)
    wave_len = (we - ws).astype(np.float64)
    # lane utilisation within a wave: mean lane time / wave time
    lane_sum = np.zeros(nw)
    np.add.at(lane_sum, wave, lane_busy)
    util = lane_sum / (64 * np.maximum(wave_len, 1))
    xcc = np.zeros(nw, np.int64)
    xcc[wave] = wt[:, 3] & 0xF
    hwid = np.zeros(nw, np.int64)
    hwid[wave] = wt[:, 2]
    end = we.max()
    tick_ns = 10.0  # s_memrealtime: 100 MHz
    print(f"waves {nw}, launch span {end * tick_ns / 1e3:.1f} us (first start -> last end)")
    print(f"last wave start at {ws.max() * tick_ns / 1e3:.1f} us; tail after it {(end - ws.max()) * tick_ns / 1e3:.1f} us")
    print(f"wave duration us: mean {wave_len.mean() * tick_ns / 1e3:.2f} p50 {np.median(wave_len) * tick_ns / 1e3:.2f} "
          f"p90 {np.percentile(wave_len, 90) * tick_ns / 1e3:.2f} max {wave_len.max() * tick_ns / 1e3:.2f}")
    pc = np.percentile(wave_len, [1, 10, 25, 50, 75, 90, 99, 99.9]) * tick_ns / 1e3
    print("wave duration percentiles 1/10/25/50/75/90/99/99.9 (us):", " ".join(f"{v:.1f}" for v in pc))
    top = np.argsort(wave_len)[-8:][::-1]
    tx = (w + 7) // 8
    print("longest waves (tile x, local tile row, us, lane util):",
          "; ".join(f"({t % tx},{t // tx}) {wave_len[t] * tick_ns / 1e3:.1f} {lane_sum[t] / (64 * max(wave_len[t], 1)):.2f}"
                    for t in top))
    print(f"lane utilisation inside waves (time-weighted): {lane_sum.sum() / (64 * wave_len.sum()):.3f}")
    # resident waves over time
    nb = 50
    edges = np.linspace(0, end, nb + 1)
    occ = []
    for i in range(nb):
        a, b = edges[i], edges[i + 1]
        ov = np.clip(np.minimum(we, b) - np.maximum(ws, a), 0, None).sum() / max(b - a, 1)
        occ.append(ov)
    print("resident waves per 2% of the span:", " ".join(f"{o:.0f}" for o in occ))
    for k in range(8):
        m = xcc == k
        if m.any():
            print(f"xcc {k}: waves {m.sum()}, last end {we[m].max() * tick_ns / 1e3:.1f} us, busy "
                  f"{wave_len[m].sum() * tick_ns / 1e3:.0f} wave-us")
    np.savez_compressed(args.out.replace(".bin", ".npz"), ws=ws, we=we, xcc=xcc, hwid=hwid, util=util)


if __name__ == "__main__":
    main()
