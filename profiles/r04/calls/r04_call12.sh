#!/bin/bash
# Round 4, call 12: the 3-ranks-on-one-GPU test repeated with its diagnostics (it failed once in
# the evidence run), then offset select (SEL) in the wavefront kernels.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "dist3_a|200|python -u -m pytest tests/test_bench_dist_gpu.py -x -q -k 'sharing_the_gpu' --timeout 150 --timeout-method thread" \
 "dist3_b|200|python -u -m pytest tests/test_bench_dist_gpu.py -x -q -k 'sharing_the_gpu' --timeout 150 --timeout-method thread" \
 "sel_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/selnb/librtamd.so python -u -m pytest tests/test_render_gpu.py tests/test_fullsize_gpu.py -x -q -k 'wavefront or fetch or c5' --timeout 250 --timeout-method thread" \
 "ab_sel|700|scripts/ab_bench.sh 'main seln selb selnb' 'c5' 2"
