#!/bin/bash
# round 5, pass c: the spectral-map kernels and the one-launch block inverse: Cayley GPU tests,
# then an alternating step A/B against the library of the previous commit; last, the queue probe
# under GPU_MAX_HW_QUEUES=2 with the native backtrace handler armed.
set -u
R=$PWD; O=$R/gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probes/pinv_probe.py 128 192 256 512 > $O/pinv.log 2>&1 || { echo probe failed; exit 1; }
grep -E "^n=|us per call" $O/pinv.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py \
    > $O/cayley.log 2>&1 || { echo "cayley tests failed"; tail -30 $O/cayley.log; exit 1; }
tail -2 $O/cayley.log
bash tools/gpu_lib_ab.sh r05c/ab 3 || exit 1
GPU_MAX_HW_QUEUES=2 timeout -k 10 240 python -u tools/probes/graph_queue_probe.py 30 4 > $O/hwq2.log 2>&1
echo "hwq2 rc=$?" | tee -a $O/hwq2.log
tail -25 $O/hwq2.log
