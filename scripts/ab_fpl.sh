#!/bin/bash
# Frames per launch at depth 1 on the final library: 4 (default) against 8 (RT_MAX_BATCH),
# C2, C3, C4, two reps.  JSON lines in gpurun_out/ab/fplN_CONFIG_REP.json.
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in c2 c3 c4; do
    for f in 4 8; do
      timeout -k 10 200 python bench.py --config $c --frames-per-launch $f --no-cpu-baseline --no-roofline --steps 480 \
          > gpurun_out/ab/fpl${f}_${c}_${r}.json 2> gpurun_out/ab/fpl${f}_${c}_${r}.err || exit 1
    done
  done
done
