#!/bin/bash
# Round 4, call 21: the persistent bounce grid (75 / 88 % of the resident blocks) re-checked with
# the 8-wave wavefront kernels, C5 interleaved.
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh "ab_grid8|400|scripts/ab_bench.sh 'main g75 g88' 'c5' 3"
