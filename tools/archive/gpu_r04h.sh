#!/bin/bash
# round 4, pass h: bench (full line with the companion configs), fan-out / cert A/B (4 vs 8 waves
# per k_lyap_fwd workgroup), the kexit probe last (it may crash at interpreter teardown)
set -u
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { rc=$?; grep -v amdgpu $O/bench.err | tail -5; exit $rc; }
cat $O/bench.json
for r in 1 2; do
  timeout -k 10 200 python tools/ab_fanout.py wg4 >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  FIODE_LIB=$PWD/tools/libfiode_fwd8.so timeout -k 10 200 python tools/ab_fanout.py wg8 >> $O/ab.jsonl 2>>$O/ab.err || exit 1
done
cat $O/ab.jsonl
timeout -k 10 200 python tools/probes/kexit_probe.py > $O/kexit.log 2>&1; echo "kexit rc=$?"; tail -12 $O/kexit.log
