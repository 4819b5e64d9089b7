#!/bin/bash
# One GPU box pass: the -m gpu suite, smoke(), then the driver's bench command.
# usage (via gpurun): bash tools/gpu_suite.sh <tag> [pytest -k expr]
set -u
TAG=${1:-r03}; K=${2:-}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" \
    > $O/suite.log 2>&1 || { echo "suite failed rc=$?"; tail -30 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
    || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
