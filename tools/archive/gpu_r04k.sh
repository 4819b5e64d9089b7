#!/bin/bash
# round 4, pass k: spread QP exit words (CONV_SLOTS) + cert batch-wise accumulation: parity, then
# the kernel trace of the throughput kernels
set -u
O=$PWD/gpurun_out/r04k; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_certify.py tests/test_gpu_lyap.py tests/test_golden.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/probes/tp_pmc.py > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
cd $R
timeout -k 10 300 python tools/ab_fanout.py > $O/ab.log 2>&1 || { echo ab failed; tail $O/ab.log; exit 1; }
tail -20 $O/ab.log
echo done
