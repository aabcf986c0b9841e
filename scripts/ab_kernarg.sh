#!/bin/bash
# A/B of where the HIP runtime puts kernel arguments (HIP_FORCE_DEV_KERNARG: unset = the
# runtime's default, 1 = device memory, 0 = host memory), C2 and C3, two reps.  JSON lines in
# gpurun_out/ab/kaV_CONFIG_REP.json.
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in c2 c3; do
    for v in def 1 0; do
      if [ $v = def ]; then
        timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 300 > gpurun_out/ab/ka${v}_${c}_${r}.json 2> gpurun_out/ab/ka${v}_${c}_${r}.err || exit 1
      else
        HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 300 > gpurun_out/ab/ka${v}_${c}_${r}.json 2> gpurun_out/ab/ka${v}_${c}_${r}.err || exit 1
      fi
    done
  done
done
