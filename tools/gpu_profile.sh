#!/bin/bash
# One GPU box pass: bench line, rocprofv3 kernel stats of the same command, and separate --pmc
# passes (MI355X_MICROARCH.md: one counter group per pass; never combined with tracing):
#   FETCH_SIZE, WRITE_SIZE                         HBM traffic per launch
#   SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES,   MFMA-busy fraction, LDS bank conflicts,
#   SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE,       kernel cycles
#   GRBM_GUI_ACTIVE
# usage (via gpurun): bash tools/gpu_profile.sh <tag> [bench args...]
set -u
TAG=${1:-r02}; shift || true
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
PMC_MFMA=""
for C in SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE; do
  if grep -q "\b$C\b" $O/counters.txt; then PMC_MFMA="$PMC_MFMA $C"; fi
done
echo "mfma pass counters:$PMC_MFMA"
for PASS in FETCH_SIZE WRITE_SIZE MFMA; do
  if [ "$PASS" = MFMA ]; then CS="$PMC_MFMA"; else CS="$PASS"; fi
  [ -z "$CS" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $O/pmc_$PASS -o run -- \
      python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-configs --prof-reps 2 > $O/pmc_$PASS.log 2>&1 || { echo "pmc $PASS failed rc=$?"; exit 1; }
done
echo done
