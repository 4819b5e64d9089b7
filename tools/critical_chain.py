"""The chain of kernels that sets one replayed step's time, read off a rocprofv3 kernel trace (not a
test).

python tools/critical_chain.py gpurun_out/<tag>/trace/run_kernel_trace.csv

Takes the same step window as tools/step_timeline.py (between two back-to-back k_ot_masks starts)
and walks back from the kernel that ends last: each link is the kernel that ended last before the
current one started (a stream / graph dependency or a full queue -- either way the current kernel
could not start earlier).  Prints the chain in time order with the idle gap in front of each
kernel, and sums the chain's busy time and gaps by kernel family.
"""
import bisect
import csv
import sys
from collections import defaultdict

from step_timeline import short


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if "k_ot_masks" in r["Kernel_Name"]]
    ts = [int(r["Start_Timestamp"]) for r in rows]
    pairs = [(a, b) for a, b in zip(starts, starts[1:])
             if 1.2e6 <= b - a <= 4e6 and bisect.bisect_left(ts, b) - bisect.bisect_left(ts, a) > 100]
    if not pairs:
        print("no back-to-back step pair found")
        return
    a, b = pairs[len(pairs) // 2]
    win = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
           for r in rows if a <= int(r["Start_Timestamp"]) < b]
    t0 = a
    cur = max(win, key=lambda k: k[1])
    chain = [cur]
    while True:
        prev = [k for k in win if k[1] <= cur[0] + 500 and k is not cur and k[0] < cur[0]]
        if not prev:
            break
        cur = max(prev, key=lambda k: k[1])
        chain.append(cur)
    chain.reverse()
    fam = defaultdict(float)
    gaps = 0.0
    last_end = None
    print(f"step window {(b - a) / 1e3:.1f} us; chain of {len(chain)} kernels")
    for s, e, n, q in chain:
        gap = 0.0 if last_end is None else max(0.0, (s - last_end) / 1e3)
        gaps += gap
        fam[n.split("<")[0].split(" ")[0][:24]] += (e - s) / 1e3
        print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  gap {gap:5.1f}  q{q}  {n}")
        last_end = e
    print(f"chain busy {sum(fam.values()):.1f} us, gaps {gaps:.1f} us")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {v:8.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
