#!/bin/bash
# Round profile of the bench workload: rocprofv3 kernel-trace stats, then the
# FETCH_SIZE / WRITE_SIZE passes (separate, counters only) for HBM traffic.
# GPU_MAX_HW_QUEUES is set here, before rocprofv3's preload starts HIP, so the profiled
# process runs with the same queue count as an unprofiled bench.py (which raises it itself).
# Outputs under gpurun_out/prof_*; summarise with scripts/profile_summary.py.
# Usage: scripts/profile_c3.sh [bench args...]   (default: the C3 headline)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$ROOT}" || exit 1
export GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- \
    python3 bench.py --steps 100 --no-cpu-baseline --no-roofline "$@" > gpurun_out/prof_trace.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- \
    python3 bench.py --steps 20 --no-cpu-baseline --no-roofline "$@" > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- \
    python3 bench.py --steps 20 --no-cpu-baseline --no-roofline "$@" > gpurun_out/prof_write.log 2>&1 || exit $?
echo done
