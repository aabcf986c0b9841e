#!/usr/bin/env python3
"""What a traversal trip costs, from a wave timeline (scripts/wave_timeline.py's .npz): a
least-squares fit of every wave's duration (start -> end of its rays) against its main-loop
trips and its wave-uniform prologue trips (scalar-cache record loads), over the waves that
ran while the chip was full (started before the first wave ended, ended before the drain).
Usage: python3 scripts/timeline_fit.py TIMELINE.npz [launch]"""
import json
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    t0, t1, t2 = (d[f"l{k}_{f}"].astype(np.float64) for f in ("t0", "t1", "t2"))
    main_, pro = d[f"l{k}_main"].astype(np.float64), d[f"l{k}_prologue"].astype(np.float64)
    dur = (t1 - t0) * 10.0   # ns
    work = (main_ + pro) > 0
    # the steady part of the launch: between the first 10 % and the last 25 % of its span
    lo, hi = t0.min() + 0.1 * (t2.max() - t0.min()), t0.min() + 0.75 * (t2.max() - t0.min())
    sel = work & (t0 >= lo) & (t1 <= hi)
    A = np.stack([main_[sel], pro[sel], np.ones(sel.sum())], 1)
    coef, res, _, _ = np.linalg.lstsq(A, dur[sel], rcond=None)
    pred = A @ coef
    r2 = 1.0 - float(((dur[sel] - pred) ** 2).sum()) / float(((dur[sel] - dur[sel].mean()) ** 2).sum())
    out = {"launch": k, "waves_fitted": int(sel.sum()), "ns_per_main_trip": round(float(coef[0]), 1),
           "ns_per_prologue_trip": round(float(coef[1]), 1), "ns_fixed_per_wave": round(float(coef[2]), 1),
           "r2": round(r2, 3), "main_trips_mean": round(float(main_[sel].mean()), 1),
           "prologue_trips_mean": round(float(pro[sel].mean()), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
