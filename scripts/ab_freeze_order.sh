#!/bin/bash
# Isolation experiment for DESIGN.md 7.5's "waves leave when done": the wave-exit epilogue (main,
# RTK_EPI_WAVE=1) and the barrier epilogue (lib/ab/b), each with the longest-first order rebuilt
# every launch and frozen after 8 launches (RTAMD_FREEZE_ORDER=8: no sort at all in the timed
# launches), plus the wave exit with a 12-entry LDS stack (lib/ab/w12).  Both knobs were experiment
# builds (profiles/r06/ab_epi_wave/epi_wave.diff + a freeze switch in render_frames); what was kept
# is RTAMD_LPT_EVERY.  The script records how profiles/r06/ab_freeze_order/ was measured.
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in c2 c3 c4; do
    for v in w wf b bf w12f; do
      lib=$PWD/real-time-opencl-raytracer_amd/lib/librtamd.so; fz=0
      case $v in wf) fz=8;; b) lib=$PWD/real-time-opencl-raytracer_amd/lib/ab/b/librtamd.so;;
                 bf) fz=8; lib=$PWD/real-time-opencl-raytracer_amd/lib/ab/b/librtamd.so;;
                 w12f) fz=8; lib=$PWD/real-time-opencl-raytracer_amd/lib/ab/w12/librtamd.so;; esac
      RTAMD_FREEZE_ORDER=$fz RTAMD_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 300 \
          > gpurun_out/ab/${v}_${c}_${r}.json 2> gpurun_out/ab/${v}_${c}_${r}.err || exit 1
    done
  done
done
