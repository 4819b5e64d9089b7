#!/bin/bash
# round 5, pass ab: graph tests (incl. the linear maps ahead), A/B of the linear maps' backward on their prefetch streams
# on each layer's stream): graph tests, then the interleaved step A/B against maps at the step start
set -u
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_graph.py \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 400 python -u tools/ab_step.py 10 default,maps_bwd_side,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
