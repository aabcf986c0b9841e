#!/bin/bash
# Round 4, call 2: the set-up fallback tests, rt_render row-group A/B, two-triangle A/B + parity,
# C2's frames-in-flight / block-order sweep.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "dist_fallback|200|python -u -m pytest tests/test_bench_dist_gpu.py -x -q -k 'unmappable or warmup' --timeout 150 --timeout-method thread" \
 "hb|500|scripts/ab_host_boundary.sh 'main g1 zc4 zc1 g3p g4pr g6p g8p g8pr g4s g6s g3s' c3 2 300" \
 "tri2_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/tri2/librtamd.so python -u -m pytest tests/test_render_gpu.py tests/test_reference_pin_gpu.py -x -q --timeout 150 --timeout-method thread" \
 "t2_parity|300|RTAMD_LIB=\$PWD/real-time-opencl-raytracer_amd/lib/ab/t2/librtamd.so python -u -m pytest tests/test_render_gpu.py tests/test_reference_pin_gpu.py -x -q --timeout 150 --timeout-method thread" \
 "ab_tri2|500|scripts/ab_bench.sh 'main tri2 tri2w7 t2 t2w6' 'c2 c3' 2" \
 "c2_inflight|300|for f in 1 2 4 8 16; do timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f > gpurun_out/r04/c2_if\$f.json || exit 1; done; for f in 4 8; do timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f --extra-flags 16 > gpurun_out/r04/c2_static_if\$f.json || exit 1; done"
