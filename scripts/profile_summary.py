"""Copies the judged profile artefacts of scripts/profile_c3.sh into profiles/<round>/
and writes profiles/<round>/pmc_<config>.json (HBM bytes per render-kernel launch).

FETCH_SIZE is doubled (gfx950 reports half the bytes of 16-B/lane reads,
MI355X_MICROARCH.md HBM section); FETCH_SIZE / WRITE_SIZE are in kB = 1024 B.

    python scripts/profile_summary.py r02 [c3] [--occupancy PMC_JSON]

--occupancy: a per-kernel summary of scripts/pmc_configs.sh, or its output directory (MeanOccupancyPerCU pass of the
same kernel, one frame in flight): its achieved waves per SIMD go into pmc_<config>.json, which
bench.py reports in roofline.occupancy.
"""
import csv
import glob
import hashlib
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# C3 is depth 1: the single-bounce kernel (FASTONLY, no next ray, the product instantiation TR = 0),
# or with bench.py's frames per launch > 1 (the depth-1 default) its batch form
KERNEL_ONE = "first_bounce_kernel<true, false, 0>"
KERNEL_BATCH = "first_bounce_batch_kernel<true, false>"
KERNEL = KERNEL_ONE


def counter(d, name):
    f = glob.glob(os.path.join(ROOT, "gpurun_out", d, "**", "*counter_collection.csv"), recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if KERNEL in r["Kernel_Name"]
         and r["Counter_Name"] == name]
    return statistics.median(v), len(v), f


def main():
    args = sys.argv[1:]
    occ_path = None
    if "--occupancy" in args:
        i = args.index("--occupancy")
        occ_path = args[i + 1]
        args = args[:i] + args[i + 2:]
    rnd = args[0] if len(args) > 0 else "r01"
    cfg = args[1] if len(args) > 1 else "c3"
    global KERNEL
    tlog = os.path.join(ROOT, "gpurun_out", "prof_trace.log")
    fpl = 1
    if os.path.exists(tlog):
        j = json.loads([ln for ln in open(tlog) if ln.startswith("{")][-1])
        fpl = int(j["config"].get("frames_per_launch", 1))
    KERNEL = KERNEL_BATCH if fpl > 1 else KERNEL_ONE
    occ = None
    if occ_path:   # a summary file, or scripts/pmc_configs.sh's output directory (the bench kernel's file in it)
        if os.path.isdir(occ_path):
            occ_path = os.path.join(occ_path, f"{cfg}_{KERNEL.split('<')[0]}.json")
        occ = json.load(open(occ_path))
    out = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(ROOT, "gpurun_out", "prof_trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(out, f"{cfg}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    # the traced run's timed window: launch order is 1 aux-count render, W warm-up frames,
    # K timed frames, then bench.py's host-boundary renders; compare with the HIP-event
    # average bench.py printed for the same K frames
    timed_us = hip_ms = None
    trace = glob.glob(os.path.join(ROOT, "gpurun_out", "prof_trace", "**", "*kernel_trace.csv"), recursive=True)
    if trace and os.path.exists(tlog):
        rows = sorted((r for r in csv.DictReader(open(trace[0])) if KERNEL in r["Kernel_Name"]),
                      key=lambda r: int(r["Start_Timestamp"]))
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        wf = j.get("warmup_frames_run", j["warmup"])   # bench.py's time-based warm-up runs more frames
        if fpl > 1:   # only the warm-up and timed frames use the batch kernel: the timed launches are the last
            t = d[-(j["steps"] // fpl):]
        else:
            t = d[1 + wf: 1 + wf + j["steps"]]
        timed_us = round(sum(t) / len(t), 2) if t else None
        hip_ms = j["roofline"].get("kernel_ms_per_launch", j["roofline"].get("kernel_ms"))
    fetch, nf, ff = counter("prof_fetch", "FETCH_SIZE")
    write, nw, fw = counter("prof_write", "WRITE_SIZE")
    shutil.copy(ff, os.path.join(out, f"{cfg}_pmc_fetch.csv"))
    shutil.copy(fw, os.path.join(out, f"{cfg}_pmc_write.csv"))
    for log in ("prof_bench.log", "prof_trace.log"):
        p = os.path.join(ROOT, "gpurun_out", log)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(out, f"{cfg}_{log.replace('prof_', '')}"))
    res = {
        "config": cfg, "kernel": "rtk_ref::" + KERNEL, "round": rnd,
        "rocprof_avg_kernel_us": None if avg_ns is None else round(avg_ns / 1e3, 2),
        "rocprof_avg_timed_window_us": timed_us,
        "hip_event_avg_timed_window_ms": hip_ms,
        "note": "rocprof_avg_kernel_us averages every launch of the traced run (warm-up, timed frames, and the "
                "one-at-a-time host-boundary renders); the timed-window average is the one bench.py reports",
        "FETCH_SIZE_kB_median": fetch, "WRITE_SIZE_kB_median": write, "dispatches": [nf, nw],
        "correction": "FETCH_SIZE x2 (gfx950 reports half the bytes of 16B/lane reads, MI355X_MICROARCH.md HBM); "
                      "kB = 1024 B",
        "hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)),
        "frames_per_launch": fpl,
        "hbm_bytes_per_frame": int(round((2 * fetch + write) * 1024 / fpl)),
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --config " + cfg,
        # the library these passes ran (the profiled tree's lib/librtamd.so; bench.py marks the
        # traffic stale when it loads a different one)
        "library_digest": hashlib.sha256(open(os.path.join(ROOT, "real-time-opencl-raytracer_amd", "lib",
                                                             "librtamd.so"), "rb").read()).hexdigest()[:16],
    }
    if occ is not None:
        d = occ["derived"]
        res["occupancy"] = {
            "waves_per_simd": round(d["waves_per_simd"], 3) if "waves_per_simd" in d else None,
            "max_waves_per_simd": 8,
            "kernel": occ["kernel"],
            "source": "rocprofv3 --pmc MeanOccupancyPerCU (SQ_LEVEL_WAVES accumulated over GRBM_GUI_ACTIVE per CU, "
                      "rocprofiler-sdk counter_defs.yaml for gfx950) / 4 SIMDs; counters are collected per dispatch, "
                      "so this is one launch alone (frames_per_launch frames), ramp-up and tail included "
                      "(scripts/pmc_configs.sh)"}
    json.dump(res, open(os.path.join(out, f"pmc_{cfg}.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
