#!/bin/bash
# r05aj: the captured step's hipGraph nodes / edges (HIP graph API)
set -o pipefail
mkdir -p gpurun_out/r05aj
timeout -k 10 300 python -u tools/probes/graph_dot_probe.py > gpurun_out/r05aj/dot.log 2>&1
