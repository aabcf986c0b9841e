#!/bin/bash
# Round 4, evidence call 2: per-frame kernel times at one frame in flight (rocprofv3 kernel
# trace) for C2-C5, occupancy + HBM + cache PMC passes for C2 and C5 (and C3), and C2's
# frames-in-flight / block-order sweep.
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
 "dist_fallback|200|python -u -m pytest tests/test_bench_dist_gpu.py -x -q -k 'unmappable or warmup' --timeout 150 --timeout-method thread" \
 "hb|300|scripts/ab_host_boundary.sh 'main g1 g3p g4pr g6p g8p g8pr' c3 2 300" \
 "trace_c2|150|trace c2" "trace_c3|150|trace c3" "trace_c4|200|trace c4" "trace_c5|300|trace c5" \
 "c2_inflight|300|for f in 1 2 4 8 16; do timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f > gpurun_out/r04/c2_if\$f.json || exit 1; done; for f in 4 8; do timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f --extra-flags 16 > gpurun_out/r04/c2_static_if\$f.json || exit 1; done" \
 "pmc_c2|400|scripts/pmc_configs.sh gpurun_out/r04/pmc c2" \
 "pmc_c5|700|scripts/pmc_configs.sh gpurun_out/r04/pmc c5"
