#!/bin/bash
# interleaved step A/B (tools/ab_step.py) + one rocprofv3 kernel trace per named variant (not a test)
# usage (via gpurun): bash tools/gpu_step_ab.sh <tag> <variants> [trace_variant ...]
set -u
export TMPDIR=/tmp
TAG=$1; V=$2; shift 2
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python tools/ab_step.py 6 $V > $O/ab.log 2>&1 || { echo ab failed; tail $O/ab.log; exit 1; }
grep "{" $O/ab.log
cd /tmp
for T in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$T -o run -- python $R/tools/ab_step.py 2 $T > $O/trace_$T.log 2>&1 || { echo trace $T failed; exit 1; }
done
echo done
