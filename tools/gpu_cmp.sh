#!/bin/bash
# Same-box kernel comparison of two trees (this one and $1): per-kernel busy time per captured step
# (tools/window_stats.py); the traces are deleted after, only the summaries come back.
set -e
O=gpurun_out/${2:-cmp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in . "$1"; do
  t=$(basename $(cd $d && pwd))
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$t -o run -- \
      python bench.py --steps 30) > $O/$t.log 2>&1
  f=$(find $O/tr_$t -name "run_kernel_trace.csv" | head -1)
  python tools/window_stats.py $f --json $O/$t.json > $O/$t.txt
  rm -rf $O/tr_$t
done
