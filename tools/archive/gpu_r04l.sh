#!/bin/bash
# round 4, pass l: k_lyap_fwd one wave per tile (both passes, one QP per lane): parity, phase probe,
# fan-out timings
set -u
O=$PWD/gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lyap.py tests/test_golden.py tests/test_gpu_sampler.py tests/test_gpu_configs.py tests/test_trajectory.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python tools/probes/lyap_probe.py > $O/lyap_probe.log 2>&1 || { echo probe failed; tail $O/lyap_probe.log; exit 1; }
cat $O/lyap_probe.log
timeout -k 10 300 python tools/ab_fanout.py > $O/ab.log 2>&1 || { echo ab failed; tail $O/ab.log; exit 1; }
tail -5 $O/ab.log
echo done
