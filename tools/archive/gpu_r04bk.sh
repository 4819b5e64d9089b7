#!/bin/bash
# round 4 (re-entry), pass bk: the small Cayley maps' loads in one round trip: Cayley tests, kernel
# stats, step A/B against the previous library
set -u
R=$PWD; O=$R/gpurun_out/r04bk; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cayley.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for L in base new; do
  if [ $L = base ]; then export FIODE_LIB=$R/tools/libfiode_base.so; else unset FIODE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$L -o run -- \
      python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/trace_$L.log 2>&1 || { echo "trace failed"; exit 1; }
  grep -h "small_cayley" $O/trace_$L/run_kernel_stats.csv | cut -c1-140
done
unset FIODE_LIB
cd $R
bash tools/gpu_lib_ab.sh r04bk/ab 3
