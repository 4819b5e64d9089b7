#!/bin/bash
# round 5, pass l: s_setprio on the GJB pivot-block elimination: spectral maps and block inverses,
# base (HEAD) vs working tree, alternating
set -u
R=$PWD; O=$R/gpurun_out/r05l; mkdir -p $O
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/new_$r.log 2>&1 || exit 1
done
for f in $O/base_1.log $O/new_1.log $O/base_2.log $O/new_2.log; do echo "== $f"; grep -v "amdgpu.ids\|^lib" $f; done
