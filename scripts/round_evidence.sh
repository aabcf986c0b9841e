#!/bin/bash
# One GPU call's worth of round-end evidence on the final library, in order: GPU test suite,
# smoke, the C3 rocprofv3 profile (kernel stats + FETCH/WRITE passes + the occupancy pass,
# summarised on the box into profiles/<round>/pmc_c3.json so the benches below read this
# library's HBM traffic and achieved waves per SIMD; copied back under gpurun_out/profiles_<round>/),
# kernel traces at one frame in flight (C3, C4, C5: per-frame kernel time against ms_per_step),
# and every config's bench line.  Each GPU step has its own time limit; a fatal step ends the
# call (scripts/gpu_steps.sh).  PMC counter sets of C2 / C5: scripts/pmc_configs.sh (own call).
# Usage: scripts/round_evidence.sh ROUND   (e.g. r04)
rnd=${1:?round}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/$rnd
export GPU_MAX_HW_QUEUES=16
trace1() {   # trace1 CONFIG: kernel trace + stats at one frame in flight
  cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
  rocprofv3 --kernel-trace --stats -d gpurun_out/$rnd/trace1_$1 -o run --output-format csv -- \
    python3 bench.py --config $1 --steps 100 --warmup 5 --inflight 1 --frames-per-launch 1 --no-cpu-baseline --no-roofline \
    > gpurun_out/$rnd/trace1_$1.json 2> gpurun_out/$rnd/trace1_$1.err
}
export -f trace1
export rnd
# SKIP_TESTS=1: the profile, traces and bench lines only (the suite and smoke in a call of their own)
tests=("pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
       "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'")
[ -n "$SKIP_TESTS" ] && tests=()
scripts/gpu_steps.sh "${tests[@]}" \
  "profile|600|scripts/profile_c3.sh && PMC_SETS=occ scripts/pmc_configs.sh gpurun_out/$rnd/pmc_occ c3 && python scripts/profile_summary.py $rnd c3 --occupancy gpurun_out/$rnd/pmc_occ && mkdir -p gpurun_out/profiles_$rnd && cp profiles/$rnd/c3_* profiles/$rnd/pmc_c3.json gpurun_out/profiles_$rnd/" \
  "trace1_c3|150|trace1 c3" "trace1_c4|200|trace1 c4" "trace1_c5|300|trace1 c5" \
  "bench_c3|240|python bench.py" \
  "bench_c3_driver|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_c1|200|python bench.py --config c1 --no-cpu-baseline" \
  "bench_c2|200|python bench.py --config c2 --no-cpu-baseline" \
  "bench_c4|240|python bench.py --config c4 --no-cpu-baseline" \
  "bench_c5|300|python bench.py --config c5 --no-cpu-baseline" \
  "bench_c5u|300|python bench.py --config c5u --no-cpu-baseline" \
  "bench_orbit|240|python bench.py --orbit 0.002 --no-cpu-baseline" \
  "bench_c3_static|240|python bench.py --jitter 1 --no-cpu-baseline"
