#!/bin/bash
# SQ counter passes over the lone block of C2's and C3's longest wave (scripts/lone_block_pmc.py),
# one rocprofv3 --pmc run per set, then the summary.  Usage: scripts/lone_pmc.sh OUT
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$ROOT}" || exit 1
out=$1; mkdir -p $out
sets=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
      "SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
      "SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
for spec in "c2 1232 608" "c3 1856 704"; do
  set -- $spec; c=$1
  i=0; mkdir -p $out/$c
  for s in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $s -d $out/$c/p$i -o run --output-format csv -- \
        python3 scripts/lone_block_pmc.py run $c $2 $3 $out/${c}_p$i.json > $out/$c/p$i.log 2>&1 || { echo "$c pass $i failed"; tail -5 $out/$c/p$i.log; exit 1; }
  done
  python3 scripts/lone_block_pmc.py summary $out/${c}_summary.json $out/$c/p* || exit 1
done
