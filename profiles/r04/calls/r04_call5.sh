#!/bin/bash
# Round 4, call 5: split-phase bounces with quad refill -- parity, C5 A/B, per-kernel trace.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
export GPU_MAX_HW_QUEUES=16
scripts/gpu_steps.sh \
 "split_parity|300|python -u -m pytest tests/test_render_gpu.py tests/test_reference_pin_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "ab_split|600|scripts/ab_bench.sh 'main nosplit lanerf rf64 rf32q' 'c5' 2" \
 "trace_c5s|200|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/r04/trace_c5s -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --inflight 1 --no-cpu-baseline --no-roofline > gpurun_out/r04/trace_c5s.json"
