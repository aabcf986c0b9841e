#!/bin/bash
# Round 4, call 18: C5's PMC counter sets again, on the library whose S_ref wavefront kernels are
# bounded to 8 waves per SIMD (the §6.3 binding table).
cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh "pmc_c5|700|scripts/pmc_configs.sh gpurun_out/r04/pmc8 c5" &&
# then the sort-chunk size re-checked with the 8-wave kernels (16 / 32 / 64 segments)
scripts/gpu_steps.sh "ab_chunk8|500|scripts/ab_bench.sh 'main ch16 ch64' 'c5' 2"
