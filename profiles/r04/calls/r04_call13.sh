#!/bin/bash
# Round 4, call 13: the GPU suite on the final tree, smoke, the driver's bench form.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "pytest_gpu|420|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench_driver|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
 "bench_default|240|python bench.py"
