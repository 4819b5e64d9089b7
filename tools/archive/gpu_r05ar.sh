#!/bin/bash
# r05ar: conv transform workgroup sizes: kernel stats of the default build and two variant builds
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05ar}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cayley.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for V in def v5 v6; do
  L=fi-ode_amd/fiode_amd/libfiode.so; [ $V != def ] && L=tools/libfiode_$V.so
  FIODE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$V -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/prof_$V.log 2>&1 || { tail -5 $O/prof_$V.log; exit 1; }
done
