#!/bin/bash
# round 4, pass g: step A/B (split with chains / split serial / one graph) under 4 / 8 / 16
# hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default is 4)
set -u
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/ab_step.py 3 split,split_serial,one_graph > $O/ab_q$q.json 2> $O/ab_q$q.err \
     || { echo "q=$q failed"; grep -v amdgpu $O/ab_q$q.err | tail -5; exit 1; }
  echo "q=$q $(cat $O/ab_q$q.json)"
done
