#!/bin/bash
# Per-rank work of an N-way band split measured on one GPU (--shard 0/N, rank 0 has the most bands),
# with rank 0's exchange work (--dist), and C2 frames in flight.  Outputs in gpurun_out/.
for n in 2 4 8; do timeout -k 10 120 python bench.py --shard 0/$n --no-cpu-baseline --no-roofline --steps 3000 > gpurun_out/shard_$n.json 2> gpurun_out/shard_$n.err || exit $?; done
timeout -k 10 120 python bench.py --dist --shard 0/8 --no-cpu-baseline --no-roofline --steps 3000 > gpurun_out/shard_8d.json 2> gpurun_out/shard_8d.err || exit $?
timeout -k 10 120 python bench.py --config c4 --shard 0/8 --no-cpu-baseline --no-roofline --steps 1000 > gpurun_out/shard_c4_8.json 2> gpurun_out/shard_c4_8.err || exit $?
for f in 2 4 8; do timeout -k 10 120 python bench.py --config c2 --inflight $f --no-cpu-baseline --no-roofline --steps 3000 > gpurun_out/c2_inflight_$f.json 2> gpurun_out/c2_inflight_$f.err || exit $?; done
