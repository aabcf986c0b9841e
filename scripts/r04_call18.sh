#!/bin/bash
# Round 4, call 18: C5's PMC counter sets again, on the library whose S_ref wavefront kernels are
# bounded to 8 waves per SIMD (the §6.3 binding table).
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh "pmc_c5|700|scripts/pmc_configs.sh gpurun_out/r04/pmc8 c5"
