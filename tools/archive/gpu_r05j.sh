#!/bin/bash
# round 5, pass j: GJB / tile LDS strides 8 mod 64 (bank-conflict-free b128 groups): spectral map and
# block inverse timings, base (HEAD~) vs working tree; correctness probe + Cayley tests
set -u
R=$PWD; O=$R/gpurun_out/r05j; mkdir -p $O
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/spec_base_$r.log 2>&1 || { echo base probe failed; tail $O/spec_base_$r.log; exit 1; }
  timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/spec_new_$r.log 2>&1 || { echo new probe failed; tail $O/spec_new_$r.log; exit 1; }
done
for f in $O/spec_*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
timeout -k 10 120 python -u tools/probes/pinv_probe.py 128 192 512 > $O/pinv.log 2>&1 || { echo pinv probe failed; exit 1; }
grep -E "^n=|chain k=3|tiles step 3" $O/pinv.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py \
    > $O/cayley.log 2>&1 || { echo "cayley tests failed"; tail -30 $O/cayley.log; exit 1; }
tail -1 $O/cayley.log
