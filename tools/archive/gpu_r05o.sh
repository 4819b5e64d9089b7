#!/bin/bash
# round 5, pass o: dopri5 forward attempt-loop phases (profiling build)
set -u
R=$PWD; O=$R/gpurun_out/r05o; mkdir -p $O
timeout -k 10 120 python -u tools/probes/odp_probe.py > $O/odp_probe.log 2>&1 || { tail $O/odp_probe.log; exit 1; }
grep -v amdgpu.ids $O/odp_probe.log
