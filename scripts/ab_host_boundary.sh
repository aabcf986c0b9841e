#!/bin/bash
# A/B of rt_render's row groups (scripts/host_boundary.py per library variant, interleaved).
# Usage: scripts/ab_host_boundary.sh "v1 v2" CONFIG REPS FRAMES
variants=$1; cfg=$2; reps=$3; frames=$4
mkdir -p gpurun_out/hb
for r in $(seq 1 "$reps"); do
  for v in $variants; do
    lib=real-time-opencl-raytracer_amd/lib/ab/$v/librtamd.so
    [ "$v" = main ] && lib=real-time-opencl-raytracer_amd/lib/librtamd.so
    RTAMD_LIB=$PWD/$lib timeout -k 10 120 python scripts/host_boundary.py "$cfg" "$frames" \
        > "gpurun_out/hb/${v}_${cfg}_${r}.json" 2> "gpurun_out/hb/${v}_${cfg}_${r}.err"
    rc=$?
    echo "$v $cfg $r rc=$rc $(cat gpurun_out/hb/${v}_${cfg}_${r}.json)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
