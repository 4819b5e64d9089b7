#!/bin/bash
# round 5, pass u: LDS bank-conflict share and MFMA busy of the inverse kernels (PMC pass over the
# spectral / block-inverse probe; never combined with tracing)
set -u
R=$PWD; O=$R/gpurun_out/r05u; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc -o run -- python $R/tools/probes/spec_probe.py > $O/pmc.log 2>&1 || { echo "pmc failed rc=$?"; tail $O/pmc.log; exit 1; }
python - $O <<'PY'
import csv, sys, glob, collections
O = sys.argv[1]
f = glob.glob(f"{O}/pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"].split("(")[0][:60]
    agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    n[(k, row["Counter_Name"])] += 1
for k, d in sorted(agg.items()):
    c, a = d.get("SQ_LDS_BANK_CONFLICT", 0), d.get("SQ_LDS_IDX_ACTIVE", 0)
    if a <= 0: continue
    print(f"{k:60s} lds conflict share {c / a:.3f}  (conflict {c:.3g} / active {a:.3g})")
PY
