#!/bin/bash
# Round 4, call 3: per-frame kernel times at one frame in flight (rocprofv3 kernel trace) for
# C2-C5, then occupancy + HBM + cache PMC passes for C2 and C5.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
export GPU_MAX_HW_QUEUES=16
trace() {   # trace CONFIG: kernel trace + stats at one frame in flight
  cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
  rocprofv3 --kernel-trace --stats -d gpurun_out/r04/trace_$1 -o run --output-format csv -- \
    python3 bench.py --config $1 --steps 100 --warmup 5 --inflight 1 --no-cpu-baseline --no-roofline \
    > gpurun_out/r04/trace_$1.json 2> gpurun_out/r04/trace_$1.err
}
export -f trace
scripts/gpu_steps.sh \
 "trace_c2|150|trace c2" "trace_c3|150|trace c3" "trace_c4|200|trace c4" "trace_c5|300|trace c5" \
 "pmc_c2|400|scripts/pmc_configs.sh gpurun_out/r04/pmc c2" \
 "pmc_c5|700|scripts/pmc_configs.sh gpurun_out/r04/pmc c5"
