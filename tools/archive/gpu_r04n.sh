#!/bin/bash
# round 4, pass n: fan-out backward phase A with one QP per lane (halves = passes): parity, phase
# probe, A/B against the HEAD build at B=128 x S=256 and B=1024 x S=1024
set -u
O=$PWD/gpurun_out/r04n; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lyap.py tests/test_golden.py tests/test_gpu_sampler.py tests/test_gpu_configs.py tests/test_trajectory.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python tools/probes/lyap_probe.py > $O/lyap_probe.log 2>&1 || { echo probe failed; tail $O/lyap_probe.log; exit 1; }
cat $O/lyap_probe.log
for i in 1 2; do
  FIODE_LIB=$R/tools/libfiode_old.so timeout -k 10 200 python tools/ab_fanout.py old --large --no-cert >> $O/ab.jsonl 2>> $O/ab.err || { echo old failed; tail $O/ab.err; exit 1; }
  timeout -k 10 200 python tools/ab_fanout.py new --large --no-cert >> $O/ab.jsonl 2>> $O/ab.err || { echo new failed; tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
echo done
