#!/bin/bash
# round 5, pass i: profile pass at HEAD (kernel stats, PMC passes) and the step's critical chain
set -u
R=$PWD
bash tools/gpu_profile.sh r05i --steps 20 --warmup 5 --no-cpu-baseline || exit 1
cd $R/tools && python critical_chain.py $R/gpurun_out/r05i/trace/run_kernel_trace.csv > $R/gpurun_out/r05i/chain.txt 2>&1 || true
head -2 $R/gpurun_out/r05i/chain.txt
