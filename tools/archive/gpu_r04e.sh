#!/bin/bash
# round 4, pass e: guard probe (which dopri5 step is skipped), split-step tests, step A/B
# (split with per-map chains / split serial / one graph), bench
set -u
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/probes/guard_probe.py > $O/guard.log 2>&1; echo "probe rc=$?"
grep -v amdgpu.ids $O/guard.log | grep -E "==|skipped [1-9]|<--" | head -20
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_graph.py tests/test_gpu_distributed.py tests/test_gpu_guard.py > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_step.py 4 default,split_serial,one_graph > $O/ab_step.json 2> $O/ab_step.err || { tail $O/ab_step.err; exit 1; }
cat $O/ab_step.json
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { rc=$?; tail -5 $O/bench.err; exit $rc; }
cat $O/bench.json
