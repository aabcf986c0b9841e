#!/usr/bin/env python3
"""How long a wave that is done waits for its block (the tile epilogue's barrier): one frame of
each config through rt_wave_timeline after warm-up frames (the product's longest-first order).

Per wave t0 = start, t1 = its pixels done, t2 = after the block epilogue.  Reports the share of
all wave-slot time (sum of t2 - t0) spent between t1 and t2 (done, holding its slot while the
block's other waves finish), and the same with the epilogue's own work taken out (t2 - max t1 of
the block: the wait is max t1 - t1).
Usage: python3 scripts/barrier_idle.py OUT.json [c2 c3 c4]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))


def run(name):
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
    for _ in range(10):
        r.render_device(w, h, depth, flags, dev.data_ptr())
    torch.cuda.synchronize()
    res = {"config": name}
    for k, tl in enumerate([r.wave_timeline(w, h, depth, flags) for _ in range(3)]):
        rec = tl["launches"][0]
        t0, t1, t2 = (rec[x].astype(np.float64) for x in ("t0", "t1", "t2"))
        ok = (t0 >= 0) & (t1 >= 0) & (t2 >= 0)
        blk = np.arange(len(t0)) // 4
        bmax = np.full(blk.max() + 1, -np.inf)
        np.maximum.at(bmax, blk[ok], t1[ok])
        slot = (t2 - t0)[ok].sum()
        wait = (bmax[blk] - t1)[ok].sum()
        res[f"run{k}"] = {"frame_ms": tl["frame_ns"] / 1e6, "waves": int(ok.sum()),
                          "share_done_to_end": round(float((t2 - t1)[ok].sum() / slot), 4),
                          "share_waiting_for_block": round(float(wait / slot), 4),
                          "mean_wave_us": round(float((t1 - t0)[ok].mean() * 10 / 1e3), 2)}
    r.close()
    return res


def main():
    out = sys.argv[1]
    res = [run(n) for n in (sys.argv[2:] or ["c2", "c3", "c4"])]
    for x in res:
        print(json.dumps(x), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
