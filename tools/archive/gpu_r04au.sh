#!/bin/bash
# round 4 (re-entry), pass au: dense maps' norm from partial sums finished in the prep kernel, the
# unit-seed Lyapunov scaling made beside the solve: Cayley / graph / train_ode tests, then the
# interleaved step A/B (tools/ab_step.py) of the two changes against their previous forms
set -u
R=$PWD; O=$R/gpurun_out/r04au; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cayley.py tests/test_gpu_graph.py tests/test_gpu_odetrain.py tests/test_gpu_optim.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python tools/ab_step.py 8 default,torch_norm,late_scale > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
