cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
for c in c5 c5u; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 bench.py --config $c --steps 50 --warmup 5 --warmup-seconds 0 --inflight 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_$c.log 2>&1 || exit $?
done
