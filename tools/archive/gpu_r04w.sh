#!/bin/bash
# round 4, pass w: kernel stats of the bench step for three builds (HEAD, 16-row parts, 32-row parts)
set -u
O=$PWD/gpurun_out/r04w; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
for v in base v32 new; do
  L=$R/tools/libfiode_$v.so; [ $v = new ] && L=$R/fi-ode_amd/fiode_amd/libfiode.so
  FIODE_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/$v.log 2>&1 || { echo $v failed; tail $O/$v.log; exit 1; }
done
echo done
