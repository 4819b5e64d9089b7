#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (not a test); usage: bash tools/gpu_trace.sh <tag>
set -u
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
echo done
