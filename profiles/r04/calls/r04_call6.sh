#!/bin/bash
# Round 4, call 6: eight work cursors for the persistent wavefront kernels -- parity, C5 A/B
# (split + quad refill, split batch, split lane refill, fused) against the round-start library.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
export GPU_MAX_HW_QUEUES=16
scripts/gpu_steps.sh \
 "cursor_parity|300|python -u -m pytest tests/test_render_gpu.py tests/test_reference_pin_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "ab_cursor|700|scripts/ab_bench.sh 'main nosplit rf64 lanerf base' 'c5' 2" \
 "trace_c5c|200|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/r04/trace_c5c -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --inflight 1 --no-cpu-baseline --no-roofline > gpurun_out/r04/trace_c5c.json"
