#!/bin/bash
# kernel trace of a short configs[1] bench and the step's critical chain (not a test)
# usage (via gpurun): bash tools/gpu_chain.sh <tag>
set -u
TAG=$1; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; tail $O/trace.log; exit 1; }
tail -1 $O/trace.log
cd $R/tools && python critical_chain.py $O/trace/run_kernel_trace.csv > $O/chain.txt 2>&1 || true
head -2 $O/chain.txt
