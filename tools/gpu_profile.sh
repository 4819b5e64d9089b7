#!/bin/bash
# One GPU box pass: bench line, rocprofv3 kernel stats of the same command, and separate
# --pmc passes for HBM traffic (FETCH_SIZE / WRITE_SIZE) of the fused kernels.
# usage (via gpurun): bash tools/gpu_profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- \
      python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --prof-reps 2 > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed rc=$?"; exit 1; }
done
echo done
