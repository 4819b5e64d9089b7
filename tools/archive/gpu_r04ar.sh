#!/bin/bash
# round 4 (re-entry), pass ar: train_ode weight-gradient chain on fewer, fuller workgroups (g_u from
# the gz1 rows, static gradients beside the slab sums): train_ode parity tests, then the step A/B
# against the HEAD library (tools/libfiode_base.so)
set -u
O=$PWD/gpurun_out/r04ar; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_lib_ab.sh r04ar/ab 2
