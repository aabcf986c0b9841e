#!/bin/bash
# Separate rocprofv3 --pmc passes (counters only, no trace domains) over a short
# bench.py run, then the median-per-dispatch summary of the render kernel.
# Usage: [BENCH_ARGS="--config c5"] scripts/pmc_c3.sh [outdir] ["COUNTER SET 1" "COUNTER SET 2" ...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$ROOT}" || exit 1
export GPU_MAX_HW_QUEUES=16
out=${1:-gpurun_out/pmc}; shift
if [ $# -eq 0 ]; then
  set -- "GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VALU" \
         "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_FLAT" \
         "FETCH_SIZE" "WRITE_SIZE"
fi
mkdir -p "$out"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set -d $out/p$i -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --warmup-seconds 0 --no-cpu-baseline --no-roofline --inflight 1 $BENCH_ARGS > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py $out/p*
