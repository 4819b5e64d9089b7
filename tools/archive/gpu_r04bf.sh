#!/bin/bash
# round 4 (re-entry), pass bf: the full GPU suite + smoke + bench at HEAD, then the profile pass
# (kernel stats, PMC HBM / MFMA passes) and the step's critical chain
set -u
R=$PWD
bash tools/gpu_suite.sh r04bf || exit 1
bash tools/gpu_profile.sh r04bg --steps 20 --warmup 5 || exit 1
cd $R/tools && python critical_chain.py $R/gpurun_out/r04bg/trace/run_kernel_trace.csv > $R/gpurun_out/r04bg/chain.txt 2>&1 || true
head -2 $R/gpurun_out/r04bg/chain.txt
