"""Summarise rocprofv3 --pmc CSVs for one kernel (median over timed dispatches).

Usage: pmc_summary.py [--kernel NAME] DIR...  (default: the C3 bench kernel, first_bounce_kernel)
"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def load(d, kernel="first_bounce_kernel"):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v[1:] if len(v) > 1 else v) for k, v in vals.items()}


if __name__ == "__main__":
    args = sys.argv[1:]
    kernel = "first_bounce_kernel"
    if args[:1] == ["--kernel"]:
        kernel, args = args[1], args[2:]
    m = {}
    for d in args:
        m.update(load(d, kernel))
    for k in sorted(m):
        print(f"{k:28s} {m[k]:16.1f}")
    g = m.get
    if g("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                print(f"  {k} / WAVE_CYCLES = {m[k] / wc:.3f}")
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        print(f"  VALU lane utilisation = {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        print(f"  L2 hit rate = {m['TCC_HIT_sum'] / max(1, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
