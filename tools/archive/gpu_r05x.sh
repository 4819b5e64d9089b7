#!/bin/bash
# round 5, pass x: the linear head's weight gradients on a side stream: tests and step A/B
set -u
R=$PWD; O=$R/gpurun_out/r05x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py -k head \
    tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_env_ab2.sh r05x/ab 3 FIODE_HEAD_WGRAD_SIDE=0 FIODE_HEAD_WGRAD_SIDE=1 || exit 1
