"""Per-step view of a rocprofv3 kernel trace of bench.py (not a test): splits the trace at the
train_ode forward launches of the captured step, and for the median step prints the busy union,
the idle gaps, and the kernels by total time.  python tools/trace_step.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"]); r["e"] = int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    r["n"] = n.split("(")[0][:48]
rows.sort(key=lambda r: r["s"])
# the graph replays: the longest run of kernels without a 30-us pause (bench.py's timed loop)
bursts, cur, end = [], [rows[0]], rows[0]["e"]
for r in rows[1:]:
    if r["s"] - end > 30000:
        bursts.append(cur)
        cur = []
    cur.append(r)
    end = max(end, r["e"])
bursts.append(cur)
rows = max(bursts, key=len)
ot = [i for i, r in enumerate(rows) if r["n"].startswith("k_ot_fwd")]
steps = []
for a, b in zip(ot, ot[1:]):
    seg = rows[a:b]
    span = (rows[b]["s"] - rows[a]["s"]) / 1e3
    steps.append((span, a, b))
steps.sort()
print("step spans (us) between consecutive k_ot_fwd:", [round(s[0]) for s in steps])
span, a, b = steps[len(steps) // 2]
seg = rows[a:b]
t0 = seg[0]["s"]
busy = 0; cur_s, cur_e = None, None; gaps = []
for r in sorted(seg, key=lambda r: r["s"]):
    if cur_e is None or r["s"] > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s; gaps.append((r["s"] - cur_e, r["n"], (cur_e - t0) / 1e3))
        cur_s, cur_e = r["s"], r["e"]
    else:
        cur_e = max(cur_e, r["e"])
busy += cur_e - cur_s
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in seg:
    tot[r["n"]] += (r["e"] - r["s"]) / 1e3; cnt[r["n"]] += 1
print(f"median step: span {span:.0f} us, {len(seg)} kernels, busy union {busy / 1e3:.0f} us, "
      f"sum of kernel times {sum(tot.values()):.0f} us, idle {span - busy / 1e3:.0f} us in {len(gaps)} gaps")
print("largest gaps (us, next kernel, at us):", [(round(g / 1e3, 1), n, round(t, 1)) for g, n, t in sorted(gaps, reverse=True)[:10]])
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:30]:
    print(f"  {t:8.1f} us  {cnt[n]:3d}x  {n}")
