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


def derived(m):
    """Ratios of one kernel's counters (medians per dispatch)."""
    g, d = m.get, {}
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                d[f"{k}/SQ_WAVE_CYCLES"] = m[k] / m["SQ_WAVE_CYCLES"]
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        d["valu_lane_utilisation"] = m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        d["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    if g("TCP_TCC_READ_REQ_sum") is not None and g("TCP_TOTAL_CACHE_ACCESSES_sum"):
        # vector L1: the share of its cache accesses that did not go on to the L2 as a read
        d["l1_hit_rate"] = 1.0 - m["TCP_TCC_READ_REQ_sum"] / m["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if g("MeanOccupancyPerCU") is not None:
        # rocprofv3's derived counter (counter_defs.yaml, gfx950: SQ_LEVEL_WAVES accumulated
        # over GRBM_GUI_ACTIVE per CU): resident waves per CU over the kernel's span; 4 SIMDs
        d["waves_per_simd"] = m["MeanOccupancyPerCU"] / 4.0
    if g("MeanOccupancyPerActiveCU") is not None:
        d["waves_per_simd_active_cu"] = m["MeanOccupancyPerActiveCU"] / 4.0
    if g("FETCH_SIZE") is not None:
        d["hbm_fetch_bytes_x2"] = 2.0 * m["FETCH_SIZE"] * 1024.0   # FETCH_SIZE in KB, x2 on gfx950 (guide)
    if g("WRITE_SIZE") is not None:
        d["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024.0
    return d


if __name__ == "__main__":
    import json
    args = sys.argv[1:]
    kernel = "first_bounce_kernel"
    out_json = None
    while args[:1] and args[0].startswith("--"):
        if args[0] == "--kernel":
            kernel, args = args[1], args[2:]
        elif args[0] == "--json":
            out_json, args = args[1], args[2:]
    m = {}
    for d in args:
        m.update(load(d, kernel))
    for k in sorted(m):
        print(f"{k:28s} {m[k]:16.1f}")
    d = derived(m)
    for k, v in d.items():
        print(f"  {k} = {v:.4g}")
    if out_json:
        json.dump({"kernel": kernel, "counters_median_per_dispatch": m, "derived": d}, open(out_json, "w"), indent=1)
