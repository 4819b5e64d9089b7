#!/bin/bash
# r05ao: stream priorities: the step captured on a high-priority stream; the ODE solve's stream at
# normal priority -- interleaved A/B, two processes
set -u
O=gpurun_out/r05ao; mkdir -p $O
for t in 1 2; do
  FIODE_PLACEMENT_TRIALS=4 timeout -k 10 500 python -u tools/ab_step.py 10 default,cap_hi,ode_lo > $O/ab_$t.json 2> $O/ab_$t.err || { tail $O/ab_$t.err; exit 1; }
  tail -1 $O/ab_$t.json
done
