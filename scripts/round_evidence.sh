#!/bin/bash
# One GPU call's worth of round-end evidence on the final library, in order:
# GPU test suite, smoke, the C3 rocprofv3 profile (kernel stats + FETCH/WRITE passes, summarised
# on the box into profiles/<round>/ so the benches below read this library's HBM traffic, copied
# back under gpurun_out/profiles_<round>/), every config's bench line, and the PMC counter sets.
# Each GPU step has its own time limit; a fatal step ends the call (scripts/gpu_steps.sh).
# Usage: scripts/round_evidence.sh ROUND   (e.g. r03)
rnd=${1:?round}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
scripts/gpu_steps.sh \
  "pytest_gpu|420|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "profile|600|scripts/profile_c3.sh && python scripts/profile_summary.py $rnd c3 && mkdir -p gpurun_out/profiles_$rnd && cp profiles/$rnd/c3_* profiles/$rnd/pmc_c3.json gpurun_out/profiles_$rnd/" \
  "bench_c3|240|python bench.py" \
  "bench_c3_driver|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_c1|200|python bench.py --config c1 --no-cpu-baseline" \
  "bench_c2|200|python bench.py --config c2 --no-cpu-baseline" \
  "bench_c4|240|python bench.py --config c4 --no-cpu-baseline" \
  "bench_c5|300|python bench.py --config c5 --no-cpu-baseline" \
  "bench_c5u|300|python bench.py --config c5u --no-cpu-baseline" \
  "bench_orbit|240|python bench.py --orbit 0.002 --no-cpu-baseline" \
  "pmc|400|scripts/pmc_c3.sh gpurun_out/pmc"
