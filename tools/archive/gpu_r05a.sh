#!/bin/bash
# round 5, pass a: the new oracle-pinning / guard tests with their printed numbers, then the full
# GPU suite + smoke + bench at HEAD
set -u
R=$PWD; O=$R/gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread \
    tests/test_gpu_odetrain_dp.py tests/test_gpu_guard.py > $O/new_tests.log 2>&1
rc=$?
tail -40 $O/new_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_suite.sh r05a_suite
