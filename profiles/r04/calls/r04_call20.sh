#!/bin/bash
# Round 4, call 20: offset select (SEL) in the depth > 1 first-bounce kernel now that it is
# scheduled for 8 waves (seln; 59 VGPRs either way): C5 parity subset, then C5 interleaved.
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh \
 "seln_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/seln/librtamd.so python -u -m pytest tests/test_render_gpu.py tests/test_fullsize_gpu.py -x -q -k 'wavefront or fetch or c5' --timeout 250 --timeout-method thread" \
 "ab_seln|500|scripts/ab_bench.sh 'main seln' 'c5 c5u' 3"
