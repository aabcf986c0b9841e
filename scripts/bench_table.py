#!/usr/bin/env python3
"""The current-numbers table of DESIGN.md from a round's bench lines (profiles/<round>/bench/*.json):
per config the rays per frame, ms per frame and Mrays/s of the timed frames (throughput mode),
the two roofline fractions, one frame alone (frame_latency), the synchronous boundary
(host_boundary, pinned), one frame per launch, and the line's file.
Usage: python3 scripts/bench_table.py [profiles/r06/bench]"""
import glob
import json
import os
import sys

ORDER = ["c1", "c2", "c3", "c3_driver", "c3_static", "orbit", "c4", "c5", "c5u"]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06/bench"
    files = {os.path.basename(f)[:-5]: f for f in glob.glob(os.path.join(d, "*.json"))}
    print("| line | rays / frame | ms / frame | Mrays/s | gather frac | latency frac | one frame alone ms | "
          "`rt_render` pinned ms | one frame per launch ms | file |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k in ORDER + sorted(set(files) - set(ORDER)):
        if k not in files:
            continue
        j = json.load(open(files[k]))
        c, r = j["config"], j["roofline"]
        g = lambda x, key: (x or {}).get(key)
        f4 = lambda v: "-" if v is None else f"{v:.4f}"
        print(f"| {k} | {c['rays_per_frame'] / 1e6:.2f} M | {j['ms_per_step']:.4f} | {j['value']:,.0f} | "
              f"{f4(r.get('frac'))} | {f4(g(r.get('latency'), 'frac'))} | {f4(g(c.get('frame_latency'), 'ms_per_frame_median'))} | "
              f"{f4(g(c.get('host_boundary'), 'ms_per_frame_pinned'))} | {f4(g(c.get('one_frame_per_launch'), 'ms_per_frame'))} | "
              f"`{files[k]}` |")


if __name__ == "__main__":
    main()
