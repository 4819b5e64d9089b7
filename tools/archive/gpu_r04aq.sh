#!/bin/bash
# round 4 (re-entry), pass aq: GPU suite + smoke + bench at HEAD, then a kernel trace of a short
# bench run for the step timeline (tools/step_timeline.py)
set -u
R=$PWD
bash tools/gpu_suite.sh r04aq || exit 1
bash tools/gpu_trace.sh r04aq_trace || exit 1
python tools/step_timeline.py $R/gpurun_out/r04aq_trace/trace/run_kernel_trace.csv --all > $R/gpurun_out/r04aq_trace/timeline.txt 2>&1 || true
head -5 $R/gpurun_out/r04aq_trace/timeline.txt
cd $R/tools && python critical_chain.py $R/gpurun_out/r04aq_trace/trace/run_kernel_trace.csv > $R/gpurun_out/r04aq_trace/chain.txt 2>&1 || true
head -3 $R/gpurun_out/r04aq_trace/chain.txt
