#!/bin/bash
# r05cd: the fused conv-1 product's X read once per (image, frequency): conv tests, then kernel stats
# of the HEAD library (tools/libfiode_base.so) and this build, alternating, k_sconv_irfft2<32, 3>
set -u
export TMPDIR=/tmp
O=gpurun_out/r05cd; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py -k "qx or spectral_conv_fused or normalized_backbone" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for V in base new; do
    L=fi-ode_amd/fiode_amd/libfiode.so; [ $V = base ] && L=tools/libfiode_base.so
    FIODE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${V}_$r -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/prof_${V}_$r.log 2>&1 || { tail -5 $O/prof_${V}_$r.log; exit 1; }
    python - "$O/prof_${V}_$r" "$V" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_sconv_irfft2<32, 3>" in r["Name"] or "k_sconv_irfft2<32>" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
  done
done
