#!/bin/bash
# round 5, pass m: dense map forward with the M-on-load one-launch inverse: tests, then the
# spectral / inverse probe (setprio) and the step A/B against the previous commit's library
set -u
R=$PWD; O=$R/gpurun_out/r05m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py \
    > $O/cayley.log 2>&1 || { echo "cayley tests failed"; tail -30 $O/cayley.log; exit 1; }
tail -1 $O/cayley.log
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/new_$r.log 2>&1 || exit 1
done
for f in $O/base_1.log $O/new_1.log $O/base_2.log $O/new_2.log; do echo "== $f"; grep -v "amdgpu.ids\|^lib" $f; done
bash tools/gpu_lib_ab.sh r05m/ab 3 || exit 1
