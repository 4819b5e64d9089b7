#!/bin/bash
# round 4 (re-entry), pass at: pipelined column-block weight gradients -- train_ode parity tests,
# kernel stats of the wgrad chain, step A/B against the HEAD library
set -u
R=$PWD; O=$R/gpurun_out/r04at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
grep -h "k_lyap_wgrad\|k_lyap_reduce\|k_lyap_static" $O/trace/run_kernel_stats.csv | cut -c1-160
cd $R
bash tools/gpu_lib_ab.sh r04at/ab 2
