#!/bin/bash
# A/B of RTAMD_LPT_EVERY (launches per rebuild of the longest-first block order): K = 1 (every
# launch), 4, 8, 16 on C2, C3, C4, C3 with an orbiting camera and C5.  JSON lines in
# gpurun_out/ab/kK_CONFIG_REP.json (scripts/ab_table.py reads them).
mkdir -p gpurun_out/ab
for r in 1 2; do
  for spec in c2 c3 c4 orbit c5; do
    c=$spec; extra=""
    [ $spec = orbit ] && { c=c3; extra="--orbit 0.002"; }
    for k in 1 4 8 16; do
      RTAMD_LPT_EVERY=$k timeout -k 10 200 python bench.py --config $c $extra --no-cpu-baseline --no-roofline --steps 300 \
          > gpurun_out/ab/k${k}_${spec}_${r}.json 2> gpurun_out/ab/k${k}_${spec}_${r}.err || exit 1
    done
  done
done
