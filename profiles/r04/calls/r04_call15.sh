#!/bin/bash
# Round 4, call 15: the GPU suite on the library whose S_ref bounce kernel is bounded to 8 waves,
# then an interleaved A/B: that library (main) vs the 7-wave bound (b7) and two LLVM scheduling
# strategies on top of main (max-ilp, max-memory-clause) on C5, C3, C2.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "pytest_gpu|420|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "ab_sched|900|scripts/ab_bench.sh 'main b7 ilp mclause' 'c5 c3 c2' 2"
