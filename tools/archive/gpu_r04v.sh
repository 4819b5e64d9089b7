#!/bin/bash
# round 4, pass v: k_lyap_wgrad staged through LDS (branch-free) with 16-row parts: train_ode parity,
# step A/B against the HEAD build
set -u
O=$PWD/gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py tests/test_gpu_graph.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 bash tools/gpu_lib_ab.sh r04v/ab 3 || exit 1
echo done
