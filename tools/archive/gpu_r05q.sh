#!/bin/bash
# round 5, pass q: solve timings, base (previous commit) against the working tree, interleaved
set -u
R=$PWD; O=$R/gpurun_out/r05q; mkdir -p $O
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/solve_ab.py > $O/solve_base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probes/solve_ab.py > $O/solve_new_$r.log 2>&1 || exit 1
done
for f in $O/solve_*.log; do echo "== $f"; grep -v "amdgpu.ids" $f; done
