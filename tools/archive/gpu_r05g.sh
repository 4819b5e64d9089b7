#!/bin/bash
# round 5, pass g: phase timestamps of the one-launch 512 inverse
set -u
R=$PWD; O=$R/gpurun_out/r05g; mkdir -p $O
timeout -k 10 120 python -u tools/probes/pinv_probe.py 512 > $O/pinv.log 2>&1 || { echo probe failed; tail $O/pinv.log; exit 1; }
grep -E "^n=|us per call|chain k|tiles step|WG start" $O/pinv.log
