#!/bin/bash
# r05ai: the captured step's hipGraph as DOT (dependency edges of the backward), the configs[2]
# guard probe (which dopri5 steps the guard skips, and why)
set -o pipefail
mkdir -p gpurun_out/r05ai
timeout -k 10 300 python -u tools/probes/graph_dot_probe.py > gpurun_out/r05ai/dot.log 2>&1 &&
timeout -k 10 300 python -u tools/probes/guard_probe.py > gpurun_out/r05ai/guard.log 2>&1
