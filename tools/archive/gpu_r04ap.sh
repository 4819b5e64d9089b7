#!/bin/bash
# round 4, pass ap: certification eta from an LDS table instead of a float64 division per value:
# parity, certification timing against the base build, kernel trace
set -u
O=$PWD/gpurun_out/r04ap; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_certify.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  FIODE_LIB=$R/tools/libfiode_base.so timeout -k 10 200 python tools/ab_fanout.py base >> $O/ab.jsonl 2>> $O/ab.err || { echo base failed; tail $O/ab.err; exit 1; }
  timeout -k 10 200 python tools/ab_fanout.py new >> $O/ab.jsonl 2>> $O/ab.err || { echo new failed; tail $O/ab.err; exit 1; }
done
python - $O/ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["tag"], d["certify_ms_per_image"], d["certify_mlp_tflops"], d["certify_max_viol"][:3])
PY
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/probes/tp_pmc.py > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo done
