"""Per-kernel busy time per captured step from a rocprofv3 kernel trace (tools; not a test).

Replay windows as tools/step_census.py defines them (k_ot_fwd4 to the next one < 2 ms later); over
the last ``--last`` windows prints the median window length and, per kernel name, the launches and
the summed duration per window (so that two trees' steps can be compared kernel by kernel).

usage: python tools/window_stats.py <kernel_trace.csv> [--last 20] [--json out.json]
"""
import argparse
import collections
import csv
import json
import statistics


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(a.trace)))
    ot = [s for s, _, n in ks if "k_ot_fwd4" in n]
    win = [(ot[i], ot[i + 1]) for i in range(len(ot) - 1) if ot[i + 1] - ot[i] < 2.0e6][-a.last:]
    per = collections.defaultdict(lambda: [0, 0.0])
    for w0, w1 in win:
        for s, e, n in ks:
            if w0 <= s < w1:
                k = n.replace("(anonymous namespace)::", "").replace("void ", "")[:90]
                per[k][0] += 1
                per[k][1] += (e - s) / 1e3
    nw = max(1, len(win))
    out = {"windows": len(win), "median_window_us": statistics.median([(b - a_) / 1e3 for a_, b in win]) if win else None,
           "kernels": {k: {"n": v[0] / nw, "us": round(v[1] / nw, 2)} for k, v in
                       sorted(per.items(), key=lambda t: -t[1][1])}}
    print(f"windows {out['windows']}  median window {out['median_window_us']:.1f} us")
    for k, v in out["kernels"].items():
        print(f"  {v['us']:9.2f} us  {v['n']:6.1f}x  {k}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
