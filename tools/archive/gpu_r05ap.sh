#!/bin/bash
# r05ap/aq: conv transforms (LDS strides, workgroup size): cayley / sconv tests, alternating bench
# A/B against the HEAD library (tools/build_base.sh), kernel stats of both
set -u
export TMPDIR=/tmp
T=${TAG:-r05ap}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cayley.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
BX=${BASEX:-}
bash tools/gpu_env_ab2.sh $T 4 "FIODE_LIB=tools/libfiode_base.so $BX" "FIODE_AB=new" || exit 1
for V in base new; do
  L=""; [ $V = base ] && L=tools/libfiode_base.so
  X=""; [ $V = base ] && X="$BX"
  env FIODE_LIB=${L:-fi-ode_amd/fiode_amd/libfiode.so} $X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$V -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/prof_$V.log 2>&1 || { tail -5 $O/prof_$V.log; exit 1; }
done
