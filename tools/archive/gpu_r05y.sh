#!/bin/bash
# round 5, pass y: interleaved A/B (one process, graphs captured first) of the linear head's
# side-stream weight gradients against autograd's head, 3 placements each
set -u
O=gpurun_out/r05y; mkdir -p $O
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 400 python -u tools/ab_step.py 10 default,head_autograd,default_b > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
