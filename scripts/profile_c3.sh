#!/bin/bash
# Round profile of the bench workload: rocprofv3 kernel-trace stats, then the
# FETCH_SIZE / WRITE_SIZE passes (separate, counters only) for HBM traffic.
# Outputs under gpurun_out/prof_*; summarise with scripts/profile_summary.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- \
    python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- \
    python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1 || exit $?
timeout -k 10 240 python3 bench.py > gpurun_out/prof_bench.log 2>&1 || exit $?
echo done
