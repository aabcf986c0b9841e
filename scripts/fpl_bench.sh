#!/bin/bash
# bench.py at several --frames-per-launch values (rt_render_device_batch), interleaved per rep;
# each JSON line in gpurun_out/fpl/CONFIG_kK_REP.json.  A run that fails stops the sweep.
# Usage: scripts/fpl_bench.sh "c2 c3" "1 2 4 8" REPS [bench args...]
configs=$1; ks=$2; reps=$3; shift 3
mkdir -p gpurun_out/fpl
for r in $(seq 1 "$reps"); do
  for c in $configs; do
    for k in $ks; do
      o=gpurun_out/fpl/${c}_k${k}_$r
      timeout -k 10 150 python bench.py --config "$c" --no-cpu-baseline --frames-per-launch "$k" "$@" > $o.json 2> $o.err
      rc=$?
      echo "$c K=$k rep $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $o.json) $(grep -o '"batch_check": {[^}]*}' $o.json)"
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
