"""Read the step graph's node / edge list (graph_dot_probe.py) against a rocprofv3 kernel trace of its
replays (not a test).

python tools/probes/graph_dot_read.py gpurun_out/graph_dot/step.json gpurun_out/<tag>/trace/run_kernel_trace.csv

Each replay's kernels are matched to the graph's kernel nodes by name, in order (node order = capture
order, trace order = start time); the match is checked against the edges (a kernel never starts
before a predecessor ends).  Per node: ready = the latest end among its graph predecessors, delay =
start - ready (time lost to the hardware queues, not to a dependency).  The critical path walks back
from the last kernel through the predecessor that set `ready`; every link prints its delay and, when
the delay is large, the kernel that ran last before it on the same queue (what it queued behind).
Medians over the replays."""
import collections
import csv
import json
import statistics
import subprocess
import sys

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from step_timeline import short  # noqa: E402


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return p.stdout.split("\n")[:len(names)]


def main(gpath, tpath):
    g = json.load(open(gpath))
    N, E = g["nodes"], g["edges"]
    kn = [n for n in N if n["type"] == 0]
    dem = demangle([n.get("name") or "?" for n in kn])
    for n, d in zip(kn, dem):
        n["short"] = short(d)
    pred = collections.defaultdict(list)
    succ = collections.defaultdict(list)
    for a, b in E:
        pred[b].append(a)
        succ[a].append(b)

    # kernel predecessors through non-kernel nodes
    def kpred(i, seen=None):
        out = []
        for p in pred[i]:
            if N[p]["type"] == 0:
                out.append(p)
            else:
                out.extend(kpred(p))
        return out
    kp = {n["i"]: sorted(set(kpred(n["i"]))) for n in kn}

    rows = list(csv.DictReader(open(tpath)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = kn[0]["short"]
    starts = [k for k, r in enumerate(rows) if short(r["Kernel_Name"]) == first]
    nk = len(kn)
    res = []
    for s in starts[-30:]:
        win = rows[s:s + 3 * nk]
        byname = collections.defaultdict(list)
        for r in win:
            byname[short(r["Kernel_Name"])].append(r)
        m = {}
        ok = True
        for n in kn:
            lst = byname.get(n["short"])
            if not lst:
                ok = False
                break
            r = lst.pop(0)
            m[n["i"]] = (int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r["Queue_Id"])
        if not ok:
            continue
        viol = sum(1 for i, ps in kp.items() for p in ps if m[i][0] < m[p][1] - 0.5)
        res.append((m, viol))
    print(f"{len(kn)} kernel nodes, {len(E)} edges, {len(res)} replays matched; "
          f"edge violations per replay {[v for _, v in res]}")
    good = [m for m, v in res if v == 0] or [m for m, _ in res]
    t0s = [min(v[0] for v in m.values()) for m in good]
    dur = {i: statistics.median(m[i][1] - m[i][0] for m in good) for i in kp}
    st = {i: statistics.median(m[i][0] - t0 for m, t0 in zip(good, t0s)) for i in kp}
    en = {i: statistics.median(m[i][1] - t0 for m, t0 in zip(good, t0s)) for i in kp}
    q = {i: collections.Counter(m[i][2] for m in good).most_common(1)[0][0] for i in kp}
    ready = {i: max((en[p] for p in kp[i]), default=0.0) for i in kp}
    span = max(en.values())
    print(f"step span (median) {span:.1f} us")
    # critical path
    cur = max(kp, key=lambda i: en[i])
    path = [cur]
    while kp[cur]:
        cur = max(kp[cur], key=lambda p: en[p])
        path.append(cur)
    path.reverse()
    tot_d = 0.0
    print(f"{'start':>8} {'dur':>6} {'delay':>6}  q  node kernel   [queued behind]")
    for i in path:
        d = st[i] - ready[i]
        tot_d += max(0.0, d)
        behind = ""
        if d > 3.0:
            same = [j for j in kp if q[j] == q[i] and en[j] <= st[i] + 1.0 and j != i]
            if same:
                b = max(same, key=lambda j: en[j])
                behind = f"[{b}:{kn_short(N, b)} ends {en[b]:.1f}]"
        print(f"{st[i]:8.1f} {dur[i]:6.1f} {d:6.1f}  q{q[i]} {i:3d} {N[i]['short'][:44]:44s} {behind}")
    print(f"critical path: {len(path)} kernels, busy {sum(dur[i] for i in path):.1f} us, "
          f"queue delays {tot_d:.1f} us")
    # graph-only bound: longest path with median durations and no queue delay
    order = sorted(kp, key=lambda i: st[i])
    lp = {}
    for i in order:
        lp[i] = dur[i] + max((lp[p] for p in kp[i]), default=0.0)
    print(f"dependency-only bound (median durations): {max(lp.values()):.1f} us")
    big = sorted(((st[i] - ready[i], i) for i in kp), reverse=True)[:15]
    print("largest delays anywhere:")
    for d, i in big:
        print(f"  {d:6.1f}  q{q[i]} {i:3d} {N[i]['short'][:50]}")


def kn_short(N, i):
    return N[i].get("short", "?")[:30]


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
