#!/bin/bash
# round 4 (re-entry), pass bc: placement selection (GraphTrainStep placement_trials): graph tests,
# the bench line (4 trials, the trial times in device_status.placement_ms), then the interleaved
# A/B of the maps' capture point with every variant's capture picked from 4 placements
set -u
R=$PWD; O=$R/gpurun_out/r04bc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['device_status'])"
FIODE_PLACEMENT_TRIALS=4 timeout -k 10 600 python tools/ab_step.py 8 default,late2,late3 > $O/ab.json 2> $O/ab.err || { echo ab failed; tail $O/ab.err; exit 1; }
cat $O/ab.json
