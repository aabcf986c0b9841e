#!/bin/bash
# Round 4, call 19: the S_ref depth-1 kernel bounded to 7 waves per SIMD (fb7: the same 59 VGPRs,
# scheduled differently) against 8 (main), interleaved on C3, C2, C4.
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh "ab_fb7|600|scripts/ab_bench.sh 'main fb7' 'c3 c2 c4' 3"
