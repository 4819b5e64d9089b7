"""MFMA-busy per dispatch from a rocprofv3 --pmc run with SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE
(not a test): busy = MFMA-busy SIMD-cycles / (GRBM_GUI_ACTIVE / XCDs x SIMDs), gfx950: 8 XCDs,
256 CUs x 4 SIMDs.  python tools/pmc_busy.py <run_counter_collection.csv> [kernel substrings...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:] or ["k_lyap_fwd", "k_lyap_bwd", "k_cert_fwd", "k_cert_final"]
d = defaultdict(lambda: defaultdict(float))
meta = {}
for r in rows:
    n = r["Kernel_Name"]
    k = next((q for q in keys if q in n), None)
    if k is None:
        continue
    d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    meta[r["Dispatch_Id"]] = (k, int(r["Grid_Size"]))
for did in sorted(d, key=int):
    c = d[did]
    k, grid = meta[did]
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024) if cyc else float("nan")
    print(f"{k:14s} grid {grid:9d}  cycles {cyc:10.0f}  MFMA-busy {busy:.3f}")
