#!/bin/bash
# round 5, pass ad: the dynamics weights' gradients as a side-stream autograd node: the solve / loss /
# graph / distributed GPU tests, then the interleaved step A/B
set -u
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py \
    tests/test_gpu_graph.py tests/test_gpu_distributed.py tests/test_gpu_guard.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 400 python -u tools/ab_step.py 10 default,dyn_wgrad_main,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
