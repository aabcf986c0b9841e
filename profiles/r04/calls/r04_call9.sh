#!/bin/bash
# Round 4, call 9: the GPU suite on 32-segment sort chunks, the A/B against 16 on C5, and the
# direction bucket count at 32-segment chunks.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "pytest_gpu|420|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "ab_chunk2|500|scripts/ab_bench.sh 'main ch16' 'c5 c5u' 2" \
 "ab_buckets|500|scripts/ab_bench.sh 'main b6 b4' 'c5' 2"
