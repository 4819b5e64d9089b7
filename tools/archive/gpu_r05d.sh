#!/bin/bash
# round 5, pass d: the one-launch block inverse stage by stage (tools/probes/pinv_probe.py)
set -u
R=$PWD; O=$R/gpurun_out/r05d; mkdir -p $O
timeout -k 10 120 python -u tools/probes/pinv_probe.py 128 192 256 512 > $O/pinv.log 2>&1; echo rc=$?
cat $O/pinv.log
