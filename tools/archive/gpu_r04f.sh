#!/bin/bash
# round 4, pass f: kernel traces of the split step and the one-graph step
set -u
O=$PWD/gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
for m in split one; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$m -o run -- \
      python $R/tools/probes/split_trace.py $m > $O/trace_$m.log 2>&1 || { echo "trace $m failed"; tail $O/trace_$m.log; exit 1; }
done
ls -R $O | head -20
