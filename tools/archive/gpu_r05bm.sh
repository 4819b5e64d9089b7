#!/bin/bash
# r05bm: Normalize fused into conv 1's transform: cayley / graph tests, then the interleaved A/B
set -u
O=gpurun_out/${TAG:-r05bm}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cayley.py tests/test_gpu_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=${TAG:-r05bm} bash tools/gpu_r05bg.sh
