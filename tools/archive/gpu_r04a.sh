#!/bin/bash
# round 4, first pass: the new guard / dopri5 / launch tests + neighbours, the bench with the
# companion lines, then the kexit probe under the native backtrace handler (last: it may crash at
# teardown)
set -u
O=gpurun_out/r04a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_guard.py tests/test_gpu_odetrain_dp.py tests/test_gpu_odetrain.py tests/test_bench_launch.py \
  tests/test_gpu_graph.py tests/test_gpu_distributed.py tests/test_gpu_optim.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { rc=$?; tail -20 $O/bench.err; exit $rc; }
cat $O/bench.json
timeout -k 10 200 python tools/probes/kexit_probe.py > $O/kexit.log 2>&1; echo "kexit rc=$?"; tail -25 $O/kexit.log
