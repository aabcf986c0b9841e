#!/usr/bin/env python3
"""Table of an ab_bench.sh run: per variant and config, ms_per_step of each rep, the one-frame
latency (frame_latency median), the synchronous boundary (host_boundary pinned) and the
one-frame-per-launch time.  Usage: python3 scripts/ab_table.py [DIR=gpurun_out/ab]"""
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
rows = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    parts = os.path.basename(f)[:-5].rsplit("_", 2)
    if len(parts) == 2:
        parts.append("1")
    v, c, r = parts
    try:
        j = json.load(open(f))
    except ValueError:
        continue
    cfg = j["config"]
    rows[(c, v)].append((j["ms_per_step"], (cfg.get("frame_latency") or {}).get("ms_per_frame_median"),
                         (cfg.get("host_boundary") or {}).get("ms_per_frame_pinned"),
                         (cfg.get("one_frame_per_launch") or {}).get("ms_per_frame")))
for (c, v), xs in sorted(rows.items()):
    col = lambda i: " ".join(f"{x[i]:.4f}" if x[i] is not None else "-" for x in xs)
    print(f"{c:4s} {v:8s} ms/step {col(0)} | frame_latency {col(1)} | host_boundary {col(2)} | 1/launch {col(3)}")
