#!/bin/bash
# round 4 (re-entry), pass bi: placement trials over more streams (maps' prefetch, ODE solve, conv
# maps computed ahead, the capture stream): graph tests, then bench lines with 4 and 8 trials
set -u
R=$PWD; O=$R/gpurun_out/r04bi; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for K in 4 8; do
  FIODE_PLACEMENT_TRIALS=$K timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-secondary > $O/bench_$K.json 2> $O/bench_$K.err || { echo bench failed; tail $O/bench_$K.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$K.json').read().strip().splitlines()[-1]); print($K, d['value'], d['ms_per_step'], d['device_status'].get('placement_ms'))"
done
