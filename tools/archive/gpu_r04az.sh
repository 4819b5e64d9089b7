#!/bin/bash
# round 4 (re-entry), pass az (second run: capture points of the maps after the first) and which side stream each linear / dynamics Cayley map is prefetched on
# (the executor placed the 4096 -> 512 map's panel chain on the step stream's hardware queue, in
# front of the conv forward): interleaved step A/B of stream assignments
set -u
R=$PWD; O=$R/gpurun_out/r04az; mkdir -p $O
timeout -k 10 600 python tools/ab_step.py 8 default,late0,late1,late3,ms_213 > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
