#!/bin/bash
# round 5, pass ae: head / conv weight gradients as side-stream tap nodes (no join): the Cayley / graph
# tests, then the interleaved A/B against the head and conv backward without the tap
set -u
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cayley.py tests/test_gpu_graph.py \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probes/graph_grad_probe.py > $O/graph_grad.log 2>&1 || { tail $O/graph_grad.log; exit 1; }
grep -c MISMATCH $O/graph_grad.log || true
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,head_autograd,conv_wgrad_main,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
