#!/bin/bash
# round 5, pass k: waves of the K = 64 real-embedding spectral inverse (GJB<128, NW>)
set -u
R=$PWD; O=$R/gpurun_out/r05k; mkdir -p $O
for nw in 16 8 4 16; do
  FIODE_SPEC_NW=$nw timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/spec_nw$nw.log 2>&1 || { echo probe failed; tail $O/spec_nw$nw.log; exit 1; }
  echo "NW=$nw: $(grep '64x256' $O/spec_nw$nw.log)"
done
