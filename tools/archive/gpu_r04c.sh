#!/bin/bash
# round 4, pass c: the split step + guard + dopri5 fixes: targeted GPU tests, the bench (full line
# with the companion configs), the fan-out / cert A/B (4 vs 8 waves), then the kexit probe (last:
# it may crash at interpreter teardown)
set -u
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_graph.py tests/test_gpu_guard.py tests/test_gpu_odetrain_dp.py tests/test_bench_launch.py \
  tests/test_gpu_certify.py tests/test_gpu_distributed.py tests/test_gpu_optim.py > $O/tests.log 2>&1
rc=$?; tail -8 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { rc=$?; tail -20 $O/bench.err; exit $rc; }
cat $O/bench.json
for r in 1 2; do
  timeout -k 10 200 python tools/ab_fanout.py wg4 >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  FIODE_LIB=$PWD/tools/libfiode_fwd8.so timeout -k 10 200 python tools/ab_fanout.py wg8 >> $O/ab.jsonl 2>>$O/ab.err || exit 1
done
cat $O/ab.jsonl
timeout -k 10 200 python tools/probes/kexit_probe.py > $O/kexit.log 2>&1; echo "kexit rc=$?"; tail -25 $O/kexit.log
