#!/bin/bash
# Round 4, call 17: round-end evidence on the library whose S_ref wavefront kernels are bounded to
# 8 waves per SIMD, then the remaining decomposition of that bound (v87: bounce kernel at 7).
cd ${GRAFT_REPO_ROOT:-.}
bash scripts/round_evidence.sh r04 && \
scripts/gpu_steps.sh "ab_waves|400|scripts/ab_bench.sh 'v88 v87 v77' 'c5' 2"
