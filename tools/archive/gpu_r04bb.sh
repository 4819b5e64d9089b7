#!/bin/bash
# round 4 (re-entry), pass bb: is the captured step's time a function of its streams?
# (tools/probes/placement_probe.py: recaptures on the same streams vs fresh pool streams)
set -u
R=$PWD; O=$R/gpurun_out/r04bb; mkdir -p $O
timeout -k 10 600 python tools/probes/placement_probe.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail $O/probe.err; exit 1; }
cat $O/probe.json
