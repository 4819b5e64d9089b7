#!/bin/bash
# round 5, pass e: which captured-graph shape the runtime's executor segfaults on under
# GPU_MAX_HW_QUEUES=2 (children per case; host faults only)
set -u
R=$PWD; O=$R/gpurun_out/r05e; mkdir -p $O
timeout -k 10 500 python -u tools/probes/hwq_branch_probe.py ${QS:-2 4} > $O/hwq_branch.log 2>&1; echo rc=$?
cat $O/hwq_branch.log
