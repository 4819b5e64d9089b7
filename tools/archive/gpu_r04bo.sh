#!/bin/bash
# round 4 (re-entry), pass bo: does the hipGraph executor release work by dependency level?
# (tools/probes/graph_level_probe.py)
set -u
R=$PWD; O=$R/gpurun_out/r04bo; mkdir -p $O
timeout -k 10 300 python tools/probes/graph_level_probe.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail $O/probe.err; exit 1; }
cat $O/probe.json
