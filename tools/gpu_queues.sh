#!/bin/bash
# step time vs the hipGraph executor's queue count (one process per setting; not a test)
set -u
export TMPDIR=/tmp
O=gpurun_out/queues; mkdir -p $O
for Q in 3 4 5 8 2 3; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$Q timeout -k 10 200 python tools/ab_step.py 4 default,conv_first > $O/q$Q.log 2>&1
  echo "Q=$Q rc=$? $(grep '{' $O/q$Q.log | cut -c1-60)"
done
