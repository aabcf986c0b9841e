#!/bin/bash
# A/B (C5, inflight 4, 1000 steps): in-tree lib vs gpurun_ab/librtamd_base.so, block order LPT (0) / static (16)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab2
for rep in 1 2; do
for v in new base; do
  for x in 0 16; do
    if [ $v = base ]; then export RTAMD_LIB=$PWD/gpurun_ab/librtamd_base.so; else unset RTAMD_LIB; fi
    timeout -k 10 200 python bench.py --config ${CFG:-c5} --no-cpu-baseline --no-roofline --steps 1000 --extra-flags $x > gpurun_out/ab2/${v}_${x}_$rep.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ab2/${v}_${x}_$rep.json'));print('$v $x $rep',d['ms_per_step'])"
  done
done
done
