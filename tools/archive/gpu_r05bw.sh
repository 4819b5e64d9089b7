#!/bin/bash
# r05bw: no zero fill / Q3 copy on the chain ahead of the solve: solve + graph tests, interleaved A/B
set -u
O=gpurun_out/r05bw; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py tests/test_gpu_graph.py tests/test_gpu_lyap.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=r05bw bash tools/gpu_r05bg.sh
