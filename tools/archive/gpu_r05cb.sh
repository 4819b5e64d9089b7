#!/bin/bash
# r05cb: conv 1's channel product fused into its inverse transform (fiode_sconv_irfft2_qx): cayley and
# graph tests, then two interleaved step A/Bs against SCONV_QX_MAX_K = 0 (fiode_cgemm + irfft2)
set -u
O=gpurun_out/r05cb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py tests/test_gpu_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,qx_off,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
