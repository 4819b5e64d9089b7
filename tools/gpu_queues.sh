#!/bin/bash
# The captured step under several graph-executor queue settings (not a test), one process each,
# with native backtraces on a host fault (tools/probes/graph_queue_probe.py).
# usage (via gpurun): bash tools/gpu_queues.sh <tag> [settings...]   ("unset" = the runtime default)
set -u
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for Q in "$@"; do
  if [ "$Q" = unset ]; then
    timeout -k 10 150 python tools/probes/graph_queue_probe.py 30 > $O/q_$Q.log 2>&1
  else
    DEBUG_HIP_FORCE_GRAPH_QUEUES=$Q timeout -k 10 150 python tools/probes/graph_queue_probe.py 30 > $O/q_$Q.log 2>&1
  fi
  rc=$?
  echo "queues=$Q rc=$rc: $(tail -1 $O/q_$Q.log)"
  # a fault, abort, time limit or any failure ends the call: nothing more runs on the GPU
  if [ $rc -ne 0 ]; then echo "stopping: rc $rc"; exit 1; fi
done
