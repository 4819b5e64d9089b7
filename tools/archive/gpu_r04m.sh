#!/bin/bash
# round 4, pass m: fan-out A/B (old: one wave per (tile, pass); new: one wave per tile, both passes)
# at B=128 x S=256 and B=1024 x S=1024, interleaved runs, then a kernel trace of the new build
set -u
O=$PWD/gpurun_out/r04m; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
for i in 1 2; do
  FIODE_LIB=$R/tools/libfiode_old.so timeout -k 10 200 python tools/ab_fanout.py old --large --no-cert >> $O/ab.jsonl 2>> $O/ab.err || { echo old failed; tail $O/ab.err; exit 1; }
  timeout -k 10 200 python tools/ab_fanout.py new --large --no-cert >> $O/ab.jsonl 2>> $O/ab.err || { echo new failed; tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/probes/tp_pmc.py > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo done
