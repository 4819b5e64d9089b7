#!/bin/bash
# Alternating bench runs under environment variants (not a test): step time and the fused kernels'
# HIP-event times per variant.  usage (via gpurun): bash tools/gpu_env_ab.sh <tag> "VAR=a" "VAR=b" ...
set -u
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for V in "$@"; do
    n=$(echo "$V" | tr '= ' '__')
    env $V timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary \
        > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { echo "bench $V failed"; tail -5 $O/bench_${n}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); k=d['roofline']['per_kernel_ms']; print('$V', d['ms_per_step'], {x: k[x] for x in ('k_lyap_bwd', 'k_lyap_reduce', 'k_lyap_fwd', 'k_ot_fwd')})"
  done
done
