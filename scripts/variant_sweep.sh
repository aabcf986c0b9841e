#!/bin/bash
# A/B sweep of kernel build variants (lib/variants/librtamd_<name>.so) over bench
# configurations; one summary line per run into gpurun_out/sweep.txt.
# Usage: scripts/variant_sweep.sh "v1 v2 ..." "label|bench args" ...
mkdir -p gpurun_out
vars="$1"; shift
for v in $vars; do
  for spec in "$@"; do
    lab="${spec%%|*}"; args="${spec#*|}"
    lib=real-time-opencl-raytracer_amd/lib/variants/librtamd_$v.so
    [ "$v" = main ] && lib=real-time-opencl-raytracer_amd/lib/librtamd.so
    RTAMD_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline $args > gpurun_out/sweep_${v}_${lab}.log 2>&1
    rc=$?
    line=$(grep '^{' gpurun_out/sweep_${v}_${lab}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" 2>/dev/null)
    echo "$v $lab rc=$rc $line" | tee -a gpurun_out/sweep.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
