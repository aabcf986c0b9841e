# A/B of the per-bounce local sort's bucket count on C5 (RTAMD_SORT_* are measurement-only knobs)
r() { name=$1; shift; env "$@" timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-roofline --steps 1000 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.log || exit 1; python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', d['ms_per_step'])"; }
r u1 RTAMD_SORT_MASK=0
r s2 RTAMD_SORT_BUCKETS=2
r s6 RTAMD_SORT_BUCKETS=6
r s8 RTAMD_SORT_BUCKETS=8
r s12 RTAMD_SORT_BUCKETS=12
r s16 RTAMD_SORT_BUCKETS=16
r s8b1 RTAMD_SORT_BUCKETS=8 RTAMD_SORT_MASK=2
r u2 RTAMD_SORT_MASK=0
r s8r RTAMD_SORT_BUCKETS=8
r s4r RTAMD_SORT_BUCKETS=4
