#!/bin/bash
# round 4 (re-entry), pass bh: earlier stream-layout variants re-measured with every capture picked
# from 4 placements (their round-3/4 A/Bs compared single captures, whose queue placement varies):
# dense maps' backward on their prefetch streams, conv map work on one shared stream, the train_ode
# solve on the step stream
set -u
R=$PWD; O=$R/gpurun_out/r04bh; mkdir -p $O
FIODE_PLACEMENT_TRIALS=4 timeout -k 10 900 python tools/ab_step.py 8 default,dense_bwd_side,conv_one_stream,ode_on_main > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
