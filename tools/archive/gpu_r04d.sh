#!/bin/bash
# round 4, pass d: the guard probe (which dopri5 step is skipped, and why), then the split-step
# tests with collectives
set -u
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/probes/guard_probe.py > $O/guard.log 2>&1; echo "probe rc=$?"
grep -v amdgpu.ids $O/guard.log | tail -70
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py tests/test_gpu_graph.py > $O/tests.log 2>&1
rc=$?; tail -8 $O/tests.log; exit $rc
