"""Busy/idle analysis of one replayed step from a rocprofv3 kernel trace (not a test)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_ot_fwd" in r["Kernel_Name"]]
# step boundaries: consecutive k_ot_fwd dispatches; take a late pair (graph replays)
cands = [(idx[i], idx[i + 1]) for i in range(len(idx) - 1) if idx[i + 1] - idx[i] > 300]
a, b = cands[len(cands) // 2]
# a step starts a bit before k_ot_fwd; use the window between two k_ot_fwd starts
win = rows[a:b]
t0, t1 = int(win[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
kt = sum(e - s for s, e in iv)
print(f"window {(t1-t0)/1e3:.1f} us, {len(win)} kernels, busy(union) {busy/1e3:.1f} us, "
      f"sum of kernel times {kt/1e3:.1f} us, queues {sorted(set(r['Queue_Id'] for r in win))}")
# distribution of gaps on the main queue
from collections import Counter
q = Counter(r["Queue_Id"] for r in win)
print("kernels per queue", dict(q))
# per-queue busy time and the main queue's biggest kernels in the window
import re
from collections import defaultdict
perq = defaultdict(float)
for r in win:
    perq[r["Queue_Id"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("busy per queue (us):", {k: round(v, 1) for k, v in sorted(perq.items())})
mainq = max(perq, key=lambda k: perq[k])
agg = defaultdict(lambda: [0, 0.0])
for r in win:
    if r["Queue_Id"] != mainq:
        continue
    n = r["Kernel_Name"]
    m = re.findall(r'(\w+Functor\w*|\w+_kernel\w*|copy_kernel|CatArray\w*|Cijk_\w{0,24}|k_\w+|reduce_kernel|fft\w{0,24}|copyBuffer|fillBuffer)', n)
    key = " ".join(dict.fromkeys(m))[:80] or n[:80]
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"main queue {mainq}: top kernels")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"  {t:8.1f} us {c:4d}x  {k}")
