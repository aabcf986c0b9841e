"""Summarise rocprofv3 --pmc CSVs for the render kernel (median over timed dispatches)."""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def load(d, kernel="render_kernel"):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v[1:] if len(v) > 1 else v) for k, v in vals.items()}


if __name__ == "__main__":
    m = {}
    for d in sys.argv[1:]:
        m.update(load(d))
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
