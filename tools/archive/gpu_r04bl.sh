#!/bin/bash
# round 4 (re-entry), pass bl: hardware queues per process (GPU_MAX_HW_QUEUES: 4 = HIP's default,
# 8, 16) with placement-picked captures (4 trials each): bench lines, alternated twice
set -u
R=$PWD; O=$R/gpurun_out/r04bl; mkdir -p $O
for i in 1 2; do
  for Q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-configs --no-secondary > $O/q${Q}_$i.json 2> $O/q${Q}_$i.err || { echo bench failed; tail $O/q${Q}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/q${Q}_$i.json').read().strip().splitlines()[-1]); print($Q, d['ms_per_step'], d['device_status'].get('placement_ms'))"
  done
done
