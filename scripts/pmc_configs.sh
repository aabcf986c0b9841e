#!/bin/bash
# PMC passes (counters only, one rocprofv3 run per set, no trace domains) of short bench.py runs
# at one frame in flight, for each config given, then per-kernel summaries (median per dispatch)
# into OUT/<config>_<kernel>.json.  Occupancy: rocprofv3's derived MeanOccupancyPerCU /
# MeanOccupancyPerActiveCU (SQ_LEVEL_WAVES); HBM: FETCH_SIZE / WRITE_SIZE.
# Usage: scripts/pmc_configs.sh OUT "c2 c5" [extra bench args...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$ROOT}" || exit 1
export GPU_MAX_HW_QUEUES=16
out=$1; cfgs=$2; shift 2
# PMC_SETS=occ: only the two occupancy passes
if [ "${PMC_SETS:-all}" = occ ]; then
  sets=("MeanOccupancyPerCU" "MeanOccupancyPerActiveCU")
else
  sets=("MeanOccupancyPerCU" "MeanOccupancyPerActiveCU" "FETCH_SIZE" "WRITE_SIZE"
        "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
        "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
        "GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum")
fi
for c in $cfgs; do
  i=0; mkdir -p "$out/$c"
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $out/$c/p$i -o run --output-format csv -- \
        python3 bench.py --config $c --steps 8 --warmup 4 --warmup-seconds 0 --no-cpu-baseline --no-roofline \
        --inflight 1 "$@" > $out/$c/p$i.log 2>&1 || { echo "$c pass $i ($set) failed"; exit 1; }
  done
  for k in first_bounce_kernel first_bounce_batch_kernel wf_bounce_kernel wf_compact_sort_kernel; do
    if grep -qs "$k" $out/$c/p1/*/*counter_collection.csv $out/$c/p1/*counter_collection.csv 2>/dev/null || \
       grep -rqs "$k" $out/$c/p1; then
      python3 scripts/pmc_summary.py --kernel $k --json $out/${c}_${k}.json $out/$c/p* > $out/${c}_${k}.txt
    fi
  done
done
