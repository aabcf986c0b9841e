#!/bin/bash
# scripts/micro/ifetch timed, then under SQ counter passes (one wave per kernel): where a lone
# wave's taken branches and mask hand-offs land among SQ_WAIT_ANY / SQ_WAIT_INST_ANY / ACTIVE.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$ROOT}" || exit 1
out=$1; mkdir -p $out
timeout -k 10 120 scripts/micro/ifetch > $out/ifetch.jsonl 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_IFETCH \
    -d $out/p1 -o run --output-format csv -- scripts/micro/ifetch 1 > $out/p1.log 2>&1 || exit 1
