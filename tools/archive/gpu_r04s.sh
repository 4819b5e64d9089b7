#!/bin/bash
# round 4, pass s: k_lyap_wgrad 16-row parts + pipelined LDS reads: parity, phase stamps, kernel stats
set -u
O=$PWD/gpurun_out/r04s; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/probes/wgrad_probe.py > $O/wgrad_probe.log 2>&1 || { echo probe failed; tail $O/wgrad_probe.log; exit 1; }
grep -v amdgpu.ids $O/wgrad_probe.log
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/new.log 2>&1 || { echo new failed; tail $O/new.log; exit 1; }
echo done
