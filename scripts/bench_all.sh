#!/bin/bash
# Every config's bench line (the tail of scripts/round_evidence.sh), each under its own limit,
# into gpurun_out/bench_<name>.log.  Usage: scripts/bench_all.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_steps.sh \
  "bench_c3|240|python bench.py" \
  "bench_c3_driver|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_c1|200|python bench.py --config c1 --no-cpu-baseline" \
  "bench_c2|200|python bench.py --config c2 --no-cpu-baseline" \
  "bench_c4|240|python bench.py --config c4 --no-cpu-baseline" \
  "bench_c5|300|python bench.py --config c5 --no-cpu-baseline" \
  "bench_c5u|300|python bench.py --config c5u --no-cpu-baseline" \
  "bench_orbit|240|python bench.py --orbit 0.002 --no-cpu-baseline"
