#!/bin/bash
# The torch-gather frame check of tests/test_bench_dist_gpu.py[6] (one rank, --dist, batches of 3
# frames, one frame per launch), repeated: with every frame's camera distinct, the assembly once read
# a set's previous contents (1 run in 6, profiles/r06/repro_dist_check/).  Usage: scripts/repro_dist_check.sh [RUNS]
mkdir -p gpurun_out/repro
n=${1:-18}
for i in $(seq 1 $n); do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29700+i)) timeout -k 10 100 python bench.py --dist --config c2 --direct --steps 4 --warmup 2 --no-cpu-baseline --cpu-seconds 0.5 --gather torch --gather-batch 3 --frames-per-launch 1 > gpurun_out/repro/t$i.json 2> gpurun_out/repro/t$i.err || exit 1
done
