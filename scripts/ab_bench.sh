#!/bin/bash
# A/B of library variants built by scripts/ab_build.sh: for each rep, config and variant
# (interleaved, so clock and box drift hit every variant alike) one bench.py run, its JSON
# line in gpurun_out/ab/VARIANT_CONFIG_REP.json.  A run that times out or crashes stops it.
# Usage: scripts/ab_bench.sh "v1 v2" "c3 c5" REPS [bench args...]
variants=$1; configs=$2; reps=$3; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 "$reps"); do
  for c in $configs; do
    for v in $variants; do
      lib=real-time-opencl-raytracer_amd/lib/ab/$v/librtamd.so
      [ "$v" = main ] && lib=real-time-opencl-raytracer_amd/lib/librtamd.so
      RTAMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config "$c" --no-cpu-baseline "$@" \
          > "gpurun_out/ab/${v}_${c}_${r}.json" 2> "gpurun_out/ab/${v}_${c}_${r}.err"
      rc=$?
      echo "$v $c $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/${v}_${c}_${r}.json)"
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
