#!/bin/bash
# Round 4, call 11: C5 at more frames in flight.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r04
scripts/gpu_steps.sh \
 "c5_inflight|600|for r in 1 2; do for f in 4 6 8; do timeout -k 5 120 python bench.py --config c5 --no-cpu-baseline --no-roofline --inflight \$f > gpurun_out/r04/c5_if\${f}_\$r.json || exit 1; echo \"c5 inflight \$f rep \$r \$(grep -o '\"ms_per_step\": [0-9.]*' gpurun_out/r04/c5_if\${f}_\$r.json)\"; done; done"
