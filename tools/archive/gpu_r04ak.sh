#!/bin/bash
# round 4, pass ak: the weight-gradient chain's slab sums + static grads in one launch: train_ode /
# graph tests, whole-step bit identity and step A/B against the HEAD build
set -u
O=$PWD/gpurun_out/r04ak; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py tests/test_gpu_graph.py tests/test_golden.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
FIODE_LIB=$PWD/tools/libfiode_base.so timeout -k 10 200 python tools/ab_params.py $O/base.pt > $O/abp.log 2>&1 || { echo abp base failed; tail $O/abp.log; exit 1; }
timeout -k 10 200 python tools/ab_params.py $O/new.pt >> $O/abp.log 2>&1 || { echo abp new failed; tail $O/abp.log; exit 1; }
python tools/ab_params.py --cmp $O/base.pt $O/new.pt; rm -f $O/base.pt $O/new.pt
timeout -k 10 900 bash tools/gpu_lib_ab.sh r04ak/ab 3 || exit 1
echo done
