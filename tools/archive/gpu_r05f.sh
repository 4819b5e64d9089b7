#!/bin/bash
# round 5, pass f: the one-launch inverse with the chain's next operands prefetched during the
# inversion, without / with the agent acquire after the polls; Cayley tests
set -u
R=$PWD; O=$R/gpurun_out/r05f; mkdir -p $O
for a in 0 1; do
  FIODE_PINV_ACQUIRE=$a timeout -k 10 120 python -u tools/probes/pinv_probe.py 128 256 512 > $O/pinv_acq$a.log 2>&1 || { echo probe failed; tail $O/pinv_acq$a.log; exit 1; }
  echo "acquire=$a"; grep -E "^n=|us per call" $O/pinv_acq$a.log
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py \
    > $O/cayley.log 2>&1 || { echo "cayley tests failed"; tail -30 $O/cayley.log; exit 1; }
tail -2 $O/cayley.log
