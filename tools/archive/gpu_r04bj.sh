#!/bin/bash
# round 4 (re-entry), pass bj: placement decision shared by the ranks: RCCL world-1 forced-comm tests
# (incl. the one-graph step picked from 3 placements) and the graph tests
set -u
R=$PWD; O=$R/gpurun_out/r04bj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_distributed.py tests/test_gpu_graph.py tests/test_bench_launch.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
