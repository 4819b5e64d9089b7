#!/bin/bash
# round 4 (re-entry), pass ba: the maps' prefetch split (the 4096 -> 512 map before the conv stack,
# the other maps after conv layer 2 / 3) against the default, each captured twice (capture-to-capture
# placement spread), interleaved
set -u
R=$PWD; O=$R/gpurun_out/r04ba; mkdir -p $O
timeout -k 10 600 python tools/ab_step.py 8 default,late3,late2,default_b,late3b > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
