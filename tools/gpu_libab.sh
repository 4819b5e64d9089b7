#!/bin/bash
# A/B of library builds on one GPU box (not a test): bit-identity of the train_ode solve against
# tools/libfiode_ref.so, then bench.py's per-kernel timing and step time with each build.
# usage (via gpurun): bash tools/gpu_libab.sh <tag> lib1.so lib2.so ...
set -u
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
FIODE_LIB=$PWD/tools/libfiode_ref.so timeout -k 10 120 python tools/ab_odetrain.py $O/ref.pt > $O/ref.log 2>&1 || { echo ref failed; exit 1; }
FIODE_LIB=$PWD/tools/libfiode_ref.so timeout -k 10 60 python tools/ab_inverse.py $O/ref_inv.pt > $O/ref_inv.log 2>&1 || { echo ref inv failed; exit 1; }
for L in "$@"; do
  n=$(basename $L .so)
  FIODE_LIB=$PWD/$L timeout -k 10 60 python tools/ab_inverse.py $O/${n}_inv.pt > $O/${n}_inv.log 2>&1 || { echo $n inv failed; tail $O/${n}_inv.log; exit 1; }
  echo "== $n inverse"; python tools/ab_inverse.py --cmp $O/ref_inv.pt $O/${n}_inv.pt
  FIODE_LIB=$PWD/$L timeout -k 10 120 python tools/ab_odetrain.py $O/$n.pt > $O/$n.log 2>&1 || { echo $n failed; tail $O/$n.log; exit 1; }
  echo "== $n"; python tools/ab_odetrain.py --cmp $O/ref.pt $O/$n.pt | grep -c identical
done
for r in 1 2; do
  for L in tools/libfiode_ref.so "$@"; do
    n=$(basename $L .so)
    FIODE_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { echo bench $n failed; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); k=d['roofline']['per_kernel_ms']; print('$n', d['ms_per_step'], 'ot_fwd', k['k_ot_fwd'], 'ot_bwd', k['k_ot_bwd+wgrad'])"
  done
done
