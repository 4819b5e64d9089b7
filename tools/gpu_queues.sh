#!/bin/bash
# step time vs the hipGraph executor's queue count (one process per setting; not a test)
set -u
export TMPDIR=/tmp
O=gpurun_out/queues; mkdir -p $O
# (6 and 8 make this ROCm runtime segfault: not run; any failure ends the script)
for Q in ${QS:-3 4 2 5}; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$Q timeout -k 10 200 python tools/ab_step.py 4 default > $O/q$Q.log 2>&1 || { echo "Q=$Q failed"; exit 1; }
  echo "Q=$Q $(grep '{' $O/q$Q.log | cut -c1-60)"
done
