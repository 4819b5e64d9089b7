#!/bin/bash
# round 4, pass q: kernel stats of the bench step, HEAD build vs the in-tree build
set -u
O=$PWD/gpurun_out/r04q; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
FIODE_LIB=$R/tools/libfiode_base.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/base.log 2>&1 || { echo base failed; tail $O/base.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/new.log 2>&1 || { echo new failed; tail $O/new.log; exit 1; }
echo done
