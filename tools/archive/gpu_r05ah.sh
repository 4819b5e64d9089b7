#!/bin/bash
# round 5, pass ah: the dense maps' backward on their forward's (prefetch) stream, after the
# dynamics-gradient tap: interleaved A/B, two processes
set -u
O=gpurun_out/r05ah; mkdir -p $O
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,dense_bwd_side,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
