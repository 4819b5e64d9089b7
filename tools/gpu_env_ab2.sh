#!/bin/bash
# Alternating configs[1] bench runs under environment variants (not a test).
# usage (via gpurun): bash tools/gpu_env_ab2.sh <tag> <rounds> "VAR=a" "VAR=b" ...
set -u
export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for V in "$@"; do
    n=$(echo "$V" | tr '= /' '___')
    env $V timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-secondary --no-configs \
        > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { echo "bench $V failed"; tail -5 $O/bench_${n}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); print('$V', d['ms_per_step'])"
  done
done
