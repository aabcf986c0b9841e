#!/bin/bash
# Round 4, call 16: which S_ref wavefront kernel gains from the 8-wave bound: vXY = depth > 1
# first-bounce kernel bounded to X waves per SIMD, bounce kernel to Y; C5 sorted and unsorted.
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh \
 "ab_waves|900|scripts/ab_bench.sh 'v88 v77 v87 v78' 'c5 c5u' 3"
