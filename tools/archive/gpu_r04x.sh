#!/bin/bash
# round 4, pass x: the captured one-graph step under GPU_MAX_HW_QUEUES 2 / 4 (default) / 8, alternating
set -u
O=$PWD/gpurun_out/r04x; mkdir -p $O
for i in 1 2; do
  for q in 2 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-configs --steps 40 --warmup 10 > $O/q${q}_$i.json 2>$O/q${q}_$i.err || { echo q$q failed; tail $O/q${q}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/q${q}_$i.json').read().strip().splitlines()[-1]); print('q$q', d['ms_per_step'])"
  done
done
