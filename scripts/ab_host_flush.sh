#!/bin/bash
# A/B of the host-memory frame path (rt_render pinned / rt_render_tiled): rtk::band_flush (default)
# against per-pixel host stores (RTAMD_HOST_FLUSH=0) and the library before it (lib/ab/prev).
# JSON lines in gpurun_out/ab/{flush,direct,prev}_CONFIG_REP.json (scripts/ab_table.py reads them).
# Rejected: the band flush and RTAMD_HOST_FLUSH were removed; the script records how
# profiles/r06/ab_host_flush/ was measured.
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in c2 c3 c4; do
    for v in flush direct prev; do
      lib=$PWD/real-time-opencl-raytracer_amd/lib/librtamd.so; env=""
      [ $v = direct ] && env="RTAMD_HOST_FLUSH=0"
      [ $v = prev ] && lib=$PWD/real-time-opencl-raytracer_amd/lib/ab/prev/librtamd.so
      env $env RTAMD_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 300 \
          > gpurun_out/ab/${v}_${c}_${r}.json 2> gpurun_out/ab/${v}_${c}_${r}.err || exit 1
    done
  done
done
