#!/bin/bash
# dopri5 train_ode + distributed GPU tests, then (only if every test passed) the atomics A/B.
set -u
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_odetrain_dp.py tests/test_gpu_distributed.py tests/test_gpu_odetrain.py \
    -v --timeout 300 --timeout-method thread > $O/dp.log 2>&1
rc=$?
tail -30 $O/dp.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit 1; fi
bash tools/gpu_env_ab.sh r03f "FIODE_DETERMINISTIC=0" "FIODE_DETERMINISTIC=1"
