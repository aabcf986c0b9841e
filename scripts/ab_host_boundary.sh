#!/bin/bash
# A/B of the synchronous boundary (scripts/host_boundary.py per variant, interleaved).  A variant
# is a library under lib/ab/NAME (main = the product library), optionally with an env setting
# after a colon: "main main:RTAMD_SYNC=block r04".
# Usage: scripts/ab_host_boundary.sh "v1 v2" CONFIG REPS FRAMES [host_boundary.py args...]
variants=$1; cfg=$2; reps=$3; frames=$4; shift 4
mkdir -p gpurun_out/hb
for r in $(seq 1 "$reps"); do
  for spec in $variants; do
    v=${spec%%:*}; envset=""; [ "$spec" != "$v" ] && envset=${spec#*:}
    lib=real-time-opencl-raytracer_amd/lib/ab/$v/librtamd.so
    [ "$v" = main ] && lib=real-time-opencl-raytracer_amd/lib/librtamd.so
    tag=$(echo "$spec" | tr ':=' '__')
    env $envset RTAMD_LIB=$PWD/$lib timeout -k 10 180 python scripts/host_boundary.py "$cfg" "$frames" "$@" \
        > "gpurun_out/hb/${tag}_${cfg}_${r}.json" 2> "gpurun_out/hb/${tag}_${cfg}_${r}.err"
    rc=$?
    echo "$spec $cfg $r rc=$rc $(cat gpurun_out/hb/${tag}_${cfg}_${r}.json)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
