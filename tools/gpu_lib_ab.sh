#!/bin/bash
# Step-time A/B of two library builds on one box (not a test): bench.py (configs[1] step only)
# alternately with tools/libfiode_base.so and the in-tree library, R rounds.
set -u
O=gpurun_out/${1:-libab}; R=${2:-2}; mkdir -p $O
for i in $(seq 1 $R); do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-configs --steps 40 --warmup 10 > $O/base_$i.json 2>/dev/null || { echo "base bench failed"; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-configs --steps 40 --warmup 10 > $O/new_$i.json 2>/dev/null || { echo "new bench failed"; exit 1; }
done
python - "$O" "$R" <<'PY'
import json, sys
O, R = sys.argv[1], int(sys.argv[2])
for k in ("base", "new"):
    v = [json.loads(open(f"{O}/{k}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, R + 1)]
    print(k, [d["ms_per_step"] for d in v])
    for d in v: print("   ", d["roofline"]["per_kernel_ms"])
PY
