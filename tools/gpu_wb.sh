#!/bin/bash
# Whole bench.py runs alternated on one box between the default and variants set by environment
# flags (the way the driver measures: a fresh process per run).
# usage (via gpurun): bash tools/gpu_wb.sh <tag> <rounds> <VAR1> [VAR2 ...]   (VAR: an env flag set to 1, or VAR=VALUE)
set -u
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for round in $(seq 1 $R); do
  for v in base "$@"; do
    i=$((i+1))
    if [ $v = base ]; then E=""; elif [[ $v == *=* ]]; then E="$v"; else E="$v=1"; fi
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-secondary \
        > $O/${i}_${v//=/-}.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$i $v done"
  done
done
