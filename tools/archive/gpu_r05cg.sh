#!/bin/bash
# r05cg: the head's output layer by fiode_head_out / _backward_gs: the GPU suite, then two interleaved
# step A/Bs against the library path (addmm, g Q3 + GroupSort backward)
set -u
O=gpurun_out/r05cg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,head_out_lib,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
