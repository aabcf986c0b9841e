#!/bin/bash
# Round 4, call 7: quad-preserving bounce sort A/B on C5 (+ its parity), lagged LPT A/B, and the
# depth-1 pin's subset sizes printed.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "sq_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/sq/librtamd.so python -u -m pytest tests/test_fullsize_gpu.py -x -q -k c5 --timeout 250 --timeout-method thread" \
 "ab_sq|500|scripts/ab_bench.sh 'main sq' 'c5' 3" \
 "lag_parity|200|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/lag/librtamd.so python -u -m pytest tests/test_render_gpu.py -x -q --timeout 150 --timeout-method thread" \
 "ab_lag|500|scripts/ab_bench.sh 'main lag' 'c3 c2 c4' 3" \
 "ab_lag_orbit|300|scripts/ab_bench.sh 'main lag' 'c3' 2 --orbit 0.002" \
 "pin_subset|300|python -u -m pytest tests/test_fullsize_gpu.py -x -q -s -k 'default_math and (c3 or c2) or c4_default' --timeout 250 --timeout-method thread"
