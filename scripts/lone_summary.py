#!/usr/bin/env python3
"""DESIGN.md 9's counter tables from profiles/r06/lone_pmc/ (scripts/lone_pmc.sh,
scripts/micro_ifetch_pmc.sh) and profiles/r06/barrier_idle/ (scripts/barrier_idle.py).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are quad-cycles (4 shader cycles): in the micro
ACTIVE_INST_VALU = INSTS_VALU, and WAVE_CYCLES x 4 = the s_memtime cycles of the loop.
Usage: python3 scripts/lone_summary.py [profiles/r06]"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def micro(d):
    timed = {}
    for l in open(os.path.join(d, "ifetch.jsonl")):
        j = json.loads(l)
        if j["waves"] == 1:
            timed.setdefault(j["variant"], []).append(j)
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Kernel_Name"].startswith("void body<"):
            per[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("micro (one wave): variant | body | cycles/inst | ACTIVE_ANY | WAIT_ANY | WAIT_INST_ANY (shares of SQ_WAVE_CYCLES)")
    order = [("add_4B", "<0, "), ("add_8B", "<1, "), ("add_4B_branch_per_8", "<2, "), ("add_8B_branch_per_8", "<3, "),
             ("add_4B_branch_over_64B_per_8", "<4, "), ("add_4B_branch_over_256B_per_8", "<5, "),
             ("add_4B_branch_over_1KB_per_8", "<6, "), ("mask_handoff_12_insts_per_8", "<7, "),
             ("exec_dance_13_insts_per_8", "<8, ")]
    for name, tag in order:
        for j in timed.get(name, []):
            k = next((k for k in per if k.startswith("void body" + tag) and k.endswith(f", {j['body_insts'] // 8}>")), None)
            sh = ""
            if k:
                m = {c: statistics.median(v) for c, v in per[k].items()}
                wc = m["SQ_WAVE_CYCLES"]
                sh = " | ".join(f"{m[c] / wc:.3f}" for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"))
            print(f"  {name:32s} {j['body_insts']:4d} | {j['cycles_per_inst']:6.2f} | {sh}")


def lone(d):
    print("\nlone block (product kernel, 16x16 window at the frame's density):")
    for c in ("c2", "c3"):
        s = json.load(open(os.path.join(d, f"{c}_summary.json")))
        w = json.load(open(os.path.join(d, f"{c}_p1.json")))
        k = next(k for k in s if "first_bounce_kernel<true, false, 0>" in k)
        m = s[k]["counters_median_per_dispatch"]
        trips = sum(x["main_trips"] + x["prologue_trips"] for x in w["waves"])
        insts = m["SQ_INSTS_VALU"] + m["SQ_INSTS_SALU"] + m["SQ_INSTS_LDS"] + m["SQ_INSTS_VMEM_RD"] + m["SQ_INSTS_BRANCH"] + m["SQ_INSTS_SMEM"]
        print(f"  {c}: waves' trips {[x['main_trips'] for x in w['waves']]} (+ prologue {sum(x['prologue_trips'] for x in w['waves'])}); "
              f"per trip: VALU {m['SQ_INSTS_VALU'] / trips:.0f}, SALU {m['SQ_INSTS_SALU'] / trips:.0f}, branches "
              f"{m['SQ_INSTS_BRANCH'] / trips:.1f}, instruction fetches {m['SQ_IFETCH'] / trips:.1f}, all {insts / trips:.0f}")
        print("      shares of SQ_WAVE_CYCLES (the block's short waves wait at the epilogue barrier inside WAIT_ANY): " +
              ", ".join(f"{c2[3:]} {v:.3f}" for c2, v in sorted(s[k]["share_of_wave_cycles"].items())))


def barrier(f):
    print("\nfull frame, one launch (rt_wave_timeline): share of wave-slot time a done wave waits for its block")
    for x in json.load(open(f)):
        r = [x[k] for k in sorted(x) if k.startswith("run")]
        print(f"  {x['config']}: waiting for the block {statistics.median(y['share_waiting_for_block'] for y in r):.3f}, "
              f"done to end (wait + epilogue) {statistics.median(y['share_done_to_end'] for y in r):.3f}, "
              f"mean wave {statistics.median(y['mean_wave_us'] for y in r):.1f} us")


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06"
    micro(os.path.join(root, "lone_pmc", "micro"))
    lone(os.path.join(root, "lone_pmc"))
    barrier(os.path.join(root, "barrier_idle", "barrier_idle.json"))
