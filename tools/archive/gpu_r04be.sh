#!/bin/bash
# round 4 (re-entry), pass be: which maps go before the conv stack (captures picked from 4
# placements, same-state trials), interleaved step A/B; graph tests for the same-state trials
set -u
R=$PWD; O=$R/gpurun_out/r04be; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
FIODE_PLACEMENT_TRIALS=4 timeout -k 10 700 python tools/ab_step.py 8 default,late1,late3,first_ab,first_dyn,late2_first_ab > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
