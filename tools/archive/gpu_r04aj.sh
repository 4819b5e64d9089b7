#!/bin/bash
# round 4, pass aj: the fused loss node's backward without the seed fill / scaling kernels:
# graph / train_ode / distributed / guard tests, then the interleaved step A/B against the round-3
# form (tools/ab_step.py old_seed)
set -u
O=$PWD/gpurun_out/r04aj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_odetrain.py tests/test_gpu_guard.py tests/test_gpu_distributed.py tests/test_gpu_configs.py tests/test_golden.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python tools/ab_step.py 4 default,old_seed > $O/ab.json 2> $O/ab.err || { echo ab failed; tail -5 $O/ab.err; exit 1; }
cat $O/ab.json
