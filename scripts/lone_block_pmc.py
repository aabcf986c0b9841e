#!/usr/bin/env python3
"""The lone block's cycles by SQ counter (what a lone-wave trip issues and
waits on, beyond DESIGN.md 9's stamps).

run CFG X0 Y0 OUT.json: the 16x16 window of CFG's frame at (X0, Y0), at the frame's pixel
density (scripts/trip_split.py window_params: the block of the frame's longest wave), rendered as
a one-block frame through the PRODUCT kernel (rt_render_device), one frame at a time with the
device idle in between, so the block's four waves have the chip (each its SIMD) to themselves.
One rt_wave_timeline frame first gives the four waves' trip counts (OUT.json).  Run it under
`rocprofv3 --pmc ...`; the one-block dispatches are the ones with Grid_Size 256.

summary OUT.json DIR...: per kernel name of the one-block dispatches, the median per dispatch of
every counter, and the split of the waves' cycles: SQ_WAIT_ANY (parked at s_waitcnt: memory, LDS,
scalar loads), SQ_WAIT_INST_ANY (ready but not issued: dependency / pipe stall), SQ_ACTIVE_INST_*
(issuing, by unit); the three add up to SQ_WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots).
"""
import csv
import glob
import json
import os
import statistics
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
FRAMES = 40


def run(name, x0, y0, out):
    import numpy as np
    import torch
    import rtamd
    from rtamd import configs
    from trip_split import window_params
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = configs.make_scene(cfg, threads=16)
    r = rtamd.Renderer(0)
    r.upload(rtamd.Scene.from_mesh(mesh, bvh))
    w, h, depth, flags = cfg["w"], cfg["h"], cfg["depth"], cfg["flags"]
    p = rtamd.params_to_array(mesh.camera_params(w, h))
    r.set_params(window_params(p, w, h, x0, y0))
    small = torch.zeros(256, dtype=torch.int32, device="cuda")
    for _ in range(10):
        r.render_device(16, 16, depth, flags, small.data_ptr())
    torch.cuda.synchronize()
    tl = r.wave_timeline(16, 16, depth, flags)["launches"][0]
    waves = [{"main_trips": int(tl["main_c"][i]), "prologue_trips": int(tl["pro_c"][i]),
              "wave_us": round(float(tl["t1"][i] - tl["t0"][i]) * 10.0 / 1e3, 2)} for i in range(len(tl["main_c"]))]
    ms = []
    for _ in range(FRAMES):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r.render_device(16, 16, depth, flags, small.data_ptr())
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t1) * 1e3)
    r.close()
    res = {"config": name, "x0": x0, "y0": y0, "frames": FRAMES, "waves": waves,
           "host_ms_per_frame_median": round(float(np.median(ms)), 4)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def summary(out, dirs):
    per = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if int(float(r.get("Grid_Size", 0))) != 256:
                    continue
                per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, vals in per.items():
        m = {c: statistics.median(v[1:] if len(v) > 1 else v) for c, v in vals.items()}
        e = {"counters_median_per_dispatch": m, "dispatches": max(len(v) for v in vals.values())}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            e["share_of_wave_cycles"] = {c: round(v / wc, 4) for c, v in m.items()
                                         if c.startswith(("SQ_WAIT", "SQ_ACTIVE_INST"))}
            if "SQ_ACTIVE_INST_ANY" in m and "SQ_INSTS_VALU" in m and "SQ_INSTS_SALU" in m:
                # instructions the block issued per quad-cycle of issuing
                e["insts_per_active_quad_cycle"] = round((m["SQ_INSTS_VALU"] + m["SQ_INSTS_SALU"]) /
                                                         m["SQ_ACTIVE_INST_ANY"], 3)
        res[k] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, e in res.items():
        print(k[:90], e["dispatches"], json.dumps(e.get("share_of_wave_cycles")))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    else:
        summary(sys.argv[2], sys.argv[3:])
