"""Compare two rocprofv3 kernel-stats CSVs (not a test): per kernel family the average duration and
calls, and the total per replay.  python tools/probes/kstats_cmp.py A.csv B.csv [pattern]"""
import csv
import re
import sys


def load(p, pat):
    d = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"]
        if pat not in n:
            continue
        m = re.search(r"(k_\w+(?:<[^>]*>)?|Cijk_\w{0,40})", n)
        k = m.group(0) if m else n[:50]
        c, t = d.get(k, (0, 0.0))
        d[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]) / 1e3)
    return d


a, b = load(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 else ""), load(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
ta = tb = 0.0
for k in sorted(set(a) | set(b), key=lambda k: -a.get(k, (1, 0))[1]):
    ca, sa = a.get(k, (0, 0.0))
    cb, sb = b.get(k, (0, 0.0))
    ta += sa
    tb += sb
    if max(sa, sb) > 100:
        print(f"{k:44s} {ca:6d} {sa / max(ca, 1):8.2f} -> {cb:6d} {sb / max(cb, 1):8.2f} us")
print(f"total {ta:.0f} -> {tb:.0f} us")
