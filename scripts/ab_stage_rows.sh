#!/bin/bash
# A/B of rtk::store_block_rows (RTAMD_STAGE_ROWS): the product default (1: host-memory frames),
# 2 (every depth-1 frame), 0 (never), and the library before it (lib/ab/prev).  JSON lines in
# gpurun_out/ab/{s1,s2,s0,prev}_CONFIG_REP.json (scripts/ab_table.py reads them).
# Rejected: the staging and RTAMD_STAGE_ROWS were removed; the script records how
# profiles/r06/ab_stage_rows/ was measured.
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in c2 c3 c4; do
    for v in s1 s2 s0 prev; do
      lib=$PWD/real-time-opencl-raytracer_amd/lib/librtamd.so; mode=1
      case $v in s2) mode=2;; s0) mode=0;; prev) lib=$PWD/real-time-opencl-raytracer_amd/lib/ab/prev/librtamd.so;; esac
      RTAMD_STAGE_ROWS=$mode RTAMD_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 300 \
          > gpurun_out/ab/${v}_${c}_${r}.json 2> gpurun_out/ab/${v}_${c}_${r}.err || exit 1
    done
  done
done
