"""One replayed training step from a rocprofv3 kernel trace, kernel by kernel (not a test).

python tools/step_timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv [--all]

A step is the window between two consecutive k_ot_masks starts that are 1.5-4 ms apart (the
back-to-back graph replays of the timed loop).  Prints per-queue busy time, the union of busy
time, and each kernel's start offset / duration / queue (kernels >= 8 us unless --all), so the
chain that sets the step time can be read off.
"""
import csv
import re
import sys
from collections import defaultdict


def short(n: str) -> str:
    m = re.findall(r"(k_\w+(?:<[^>]*>)?|Cijk_\w{0,28}|\w+Functor\w*|reduce_kernel|copyBuffer\w*|fillBuffer\w*|"
                   r"CatArray\w*|multi_tensor_apply_kernel)", n)
    return (" ".join(dict.fromkeys(m)) or n)[:60]


def main(path, show_all=False):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if "k_ot_masks" in r["Kernel_Name"]]
    ts = [int(r["Start_Timestamp"]) for r in rows]
    import bisect
    pairs = [(a, b) for a, b in zip(starts, starts[1:])
             if 1.5e6 <= b - a <= 4e6 and bisect.bisect_left(ts, b) - bisect.bisect_left(ts, a) > 100]
    if not pairs:
        print("no back-to-back step pair found")
        return
    a, b = pairs[len(pairs) // 2]
    pre = 150_000                      # the step's first kernels run ahead of k_ot_masks
    win = [r for r in rows if a - pre <= int(r["Start_Timestamp"]) < b - pre]
    t0 = min(int(r["Start_Timestamp"]) for r in win)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    perq = defaultdict(float)
    for r in win:
        perq[r["Queue_Id"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"step window {(b - a) / 1e3:.1f} us, {len(win)} kernels, busy(union) {busy / 1e3:.1f} us, "
          f"sum {sum(perq.values()):.1f} us")
    print("busy per queue (us):", {k: round(v, 1) for k, v in sorted(perq.items())})
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        if show_all or d >= 8.0:
            print(f"  q{r['Queue_Id']} {(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f}  {d:7.1f}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], "--all" in sys.argv)
