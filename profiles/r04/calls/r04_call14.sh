#!/bin/bash
# Round 4, call 14: C5's persistent bounce grid (50/75/150 % of the resident blocks) and an
# 8-wave bound for the wavefront kernels, interleaved; then frames in flight 2/3/5 on C5.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
inflight() {
  for r in 1 2; do for n in 2 3 4 5; do
    timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --inflight $n > gpurun_out/r04/c5_if${n}_$r.json 2>/dev/null || return 1
    echo "c5 inflight $n rep $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04/c5_if${n}_$r.json)"
  done; done
}
export -f inflight
scripts/gpu_steps.sh \
 "ab_grid|600|scripts/ab_bench.sh 'main g50 g75 g150 w8' 'c5' 2" \
 "c5_inflight|400|inflight"
