#!/bin/bash
# A/B over library variants: LIBS="name ..." (cur = in-tree, else gpurun_ab/librtamd_<name>.so); CFG, EXTRA
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for rep in 1 2; do
  for v in ${LIBS:-cur}; do
    if [ $v = cur ]; then unset RTAMD_LIB; else export RTAMD_LIB=$PWD/gpurun_ab/librtamd_$v.so; fi
    timeout -k 10 200 python bench.py --config ${CFG:-c5} --no-cpu-baseline --no-roofline --steps ${STEPS:-1000} $EXTRA > gpurun_out/abl/${v}_$rep.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/abl/${v}_$rep.json'));print('$v $rep',d['ms_per_step'])"
  done
done
