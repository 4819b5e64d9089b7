#!/bin/bash
# round 4 (re-entry), pass as: profile pass of the column-block weight-gradient chain (bench line,
# kernel stats, PMC HBM / MFMA passes via tools/gpu_profile.sh), the base library's kernel stats
# beside it, and the step's critical chain from the trace
set -u
R=$PWD; O=$R/gpurun_out/r04as; mkdir -p $O
bash tools/gpu_profile.sh r04as --steps 20 --warmup 5 || exit 1
cd /tmp
FIODE_LIB=$R/tools/libfiode_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base_trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/base_trace.log 2>&1 || { echo "base trace failed"; exit 1; }
cd $R/tools
python critical_chain.py $O/trace/run_kernel_trace.csv > $O/chain.txt 2>&1 || true
python step_timeline.py $O/trace/run_kernel_trace.csv --all > $O/timeline.txt 2>&1 || true
head -3 $O/chain.txt
grep -h "k_lyap_wgrad\|k_lyap_reduce\|k_lyap_static" $O/trace/run_kernel_stats.csv $O/base_trace/run_kernel_stats.csv | cut -c1-200
