#!/bin/bash
# round 5, pass z: the conv layers' weight / bias gradients on the side stream: the conv gradient
# tests, then the interleaved step A/B against the single-stream conv backward
set -u
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py -k "spectral_conv or head or spatial_major" \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 400 python -u tools/ab_step.py 10 default,conv_wgrad_main,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
