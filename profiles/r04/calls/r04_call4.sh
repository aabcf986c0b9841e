#!/bin/bash
# Round 4, call 4: split-phase refilling bounces (RTK_SPLIT) -- parity, then C5 A/B against the
# fused bounce kernel; C2 at more frames in flight (16 frame slots).
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "split_parity|400|python -u -m pytest tests/test_render_gpu.py tests/test_reference_pin_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "ab_split|500|scripts/ab_bench.sh 'main nosplit rf8 rf32' 'c5' 2" \
 "inflight|400|for f in 6 8 12 16; do timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f > gpurun_out/r04/c2b_if\$f.json || exit 1; timeout -k 5 60 python bench.py --config c2 --no-cpu-baseline --no-roofline --inflight \$f --extra-flags 16 > gpurun_out/r04/c2b_static_if\$f.json || exit 1; done; for f in 8 12; do timeout -k 5 60 python bench.py --config c3 --no-cpu-baseline --no-roofline --inflight \$f > gpurun_out/r04/c3b_if\$f.json || exit 1; done"
