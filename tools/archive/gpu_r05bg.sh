#!/bin/bash
# r05bg: where the late maps' prefetch is captured, after the round-5 conv stack: interleaved A/B
set -u
O=gpurun_out/${TAG:-r05bg}; mkdir -p $O
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,pre_solve_old,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
