#!/bin/bash
# Round 4, call 8: bounce-queue sort chunk size A/B on C5 (+ parity of the largest).
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "ch_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/ch64/librtamd.so python -u -m pytest tests/test_render_gpu.py -x -q -k 'wavefront or fetch' --timeout 150 --timeout-method thread" \
 "ab_chunk|600|scripts/ab_bench.sh 'main ch8 ch32 ch64' 'c5' 2"
