"""Per-frame kernel time of a rocprofv3 --kernel-trace run of bench.py at one frame in flight,
set against the ms_per_step the same run printed.

The traced bench.py launches, in order: one aux render (ray counts), the warm-up frames
(`warmup_frames_run`), the `steps` timed frames, then the host-boundary renders.  A frame is
`kernels_per_frame` launches of the library's render kernels (rtk_*: 1 at depth 1; C5: first
bounce + 2 x (compaction + bounce)).  For the timed frames: the sum of their kernels' durations
and the span from the first kernel's start to the last one's end, both per frame.

    python scripts/trace_summary.py TRACE_DIR BENCH_JSON [OUT_JSON]
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    tdir, bjson = sys.argv[1], sys.argv[2]
    j = json.loads([ln for ln in open(bjson) if ln.startswith("{")][-1])
    depth = j["config"]["depth"]
    wavefront = bool(j["config"]["flags"] & 8) or depth == 1
    kpf = 1 if depth == 1 else (1 + 2 * (depth - 1) if wavefront else 1)
    f = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((r for r in csv.DictReader(open(f)) if "rtk" in r["Kernel_Name"] and "peak" not in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    wf = j.get("warmup_frames_run", j["warmup"])
    first = (1 + wf) * kpf
    timed = rows[first: first + j["steps"] * kpf]
    frames = [timed[i:i + kpf] for i in range(0, len(timed), kpf)]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fr) / 1e6 for fr in frames]
    span = [(int(fr[-1]["End_Timestamp"]) - int(fr[0]["Start_Timestamp"])) / 1e6 for fr in frames]
    per_kernel = {}
    for fr in frames:
        for i, r in enumerate(fr):
            n = f"{i}: " + r["Kernel_Name"].split("(")[0]
            per_kernel.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {"config": j["config"]["config"], "frames_in_flight": j["config"]["frames_in_flight"],
           "timed_frames": len(frames), "kernels_per_frame": kpf,
           "ms_per_step": j["ms_per_step"],
           "kernel_ms_per_frame_mean": round(statistics.mean(busy), 4),
           "kernel_span_ms_per_frame_mean": round(statistics.mean(span), 4),
           "kernel_ms_le_frame_ms": statistics.mean(busy) <= j["ms_per_step"],
           "per_kernel_us_mean": {k: round(statistics.mean(v), 1) for k, v in per_kernel.items()},
           "source": os.path.relpath(f)}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
