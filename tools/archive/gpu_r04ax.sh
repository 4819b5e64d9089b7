#!/bin/bash
# round 4 (re-entry), pass ax: the full GPU suite + smoke + bench at HEAD, then the profile pass
# (kernel stats, PMC HBM / MFMA passes) and the step's critical chain
set -u
R=$PWD
bash tools/gpu_suite.sh r04ax || exit 1
bash tools/gpu_profile.sh r04ay --steps 20 --warmup 5 || exit 1
cd $R/tools && python critical_chain.py $R/gpurun_out/r04ay/trace/run_kernel_trace.csv > $R/gpurun_out/r04ay/chain.txt 2>&1 || true
head -2 $R/gpurun_out/r04ay/chain.txt
