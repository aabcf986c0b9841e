#!/bin/bash
# Round 4, call 10: first-bounce queue order in bands of tile rows (RTK_SEG_BAND) on C5.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "band_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/band4/librtamd.so python -u -m pytest tests/test_render_gpu.py tests/test_fullsize_gpu.py -x -q -k 'wavefront or fetch or c5' --timeout 250 --timeout-method thread" \
 "ab_band|600|scripts/ab_bench.sh 'main band2 band4 band8' 'c5' 2"
