"""Longest dependency path of the captured training step (tools; not a test).

Reads the step's hipGraph as DOT (tools/probes/graph_dag_probe.py: kernel nodes, launch shapes and
edges) and a rocprofv3 kernel trace of the same process's replays, gives every graph node its
kernels' median duration over the replay windows (matched by demangled name + launch shape +
occurrence order), and prints:
  * the longest path through the DAG with those durations -- the step time if every kernel started
    the moment its dependencies ended (no queue, dispatch or contention effects);
  * the measured replay window, and for the last window each node's "late start": its start minus
    the latest end of its graph predecessors (time it could have run but did not), largest first.

usage: python tools/dag_critical.py gpurun_out/<tag>/step.dot gpurun_out/<tag>/trace/run_kernel_trace.csv
"""
import collections
import csv
import re
import statistics
import subprocess
import sys


def demangle(names):
    tool = "c++filt"
    try:
        out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except Exception:                     # noqa: BLE001 - fall back to the raw names
        return list(names)


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def main(dot, trace):
    txt = open(dot).read()
    nodes = {}
    for m in re.finditer(r'"graph_\d+_node_(\d+)"\[style="\w+"shape="record"label="\{\n(\w+)\n(.*?)\}"\];', txt, re.S):
        nid, kind, body = int(m.group(1)), m.group(2), m.group(3)
        name, grid, block = None, None, None
        k = re.search(r"\{ID \| \d+ \| (.*?)\\<\\<\\<\((\d+),(\d+),(\d+)\),\((\d+),(\d+),(\d+)\)", body)
        if k:
            name = k.group(1)
            grid = tuple(int(k.group(i)) for i in (2, 3, 4))
            block = tuple(int(k.group(i)) for i in (5, 6, 7))
        nodes[nid] = {"kind": kind, "name": name, "grid": grid, "block": block}
    edges = [(int(a), int(b)) for a, b in re.findall(r'"graph_\d+_node_(\d+)" -> "graph_\d+_node_(\d+)"', txt)]
    kn = [i for i in sorted(nodes) if nodes[i]["name"]]
    dem = demangle([nodes[i]["name"] for i in kn])
    for i, d in zip(kn, dem):
        nodes[i]["dname"] = d
    preds = collections.defaultdict(list)
    succ = collections.defaultdict(list)
    for a, b in edges:
        preds[b].append(a)
        succ[a].append(b)
    # topological order
    indeg = {i: len(preds[i]) for i in nodes}
    order, q = [], [i for i in sorted(nodes) if indeg[i] == 0]
    while q:
        i = q.pop(0)
        order.append(i)
        for j in succ[i]:
            indeg[j] -= 1
            if indeg[j] == 0:
                q.append(j)
    rows = list(csv.DictReader(open(trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])),
                 (int(r["Workgroup_Size_X"]), int(r["Workgroup_Size_Y"]), int(r["Workgroup_Size_Z"])), r["Queue_Id"])
                for r in rows)
    key = lambda name, grid, block: (short(name), tuple(g * b for g, b in zip(grid, block)), block)  # noqa: E731
    # replay windows: from one launch of a root kernel that occurs once per graph to the next
    cnt = collections.Counter(key(nodes[i]["dname"], nodes[i]["grid"], nodes[i]["block"])
                              for i in order if nodes[i].get("name"))
    root = next(i for i in order if nodes[i].get("name") and not preds[i]
                and cnt[key(nodes[i]["dname"], nodes[i]["grid"], nodes[i]["block"])] == 1)
    rk = key(nodes[root]["dname"], nodes[root]["grid"], nodes[root]["block"])
    ot = [s for s, _, n, g, bl, _ in ks if (short(n), g, bl) == rk]
    wins = [(ot[i], ot[i + 1]) for i in range(len(ot) - 1) if ot[i + 1] - ot[i] < 3.0e6]
    per_win = []
    for a, b in wins:
        bucket = collections.defaultdict(list)
        for s, e, n, g, bl, qid in ks:
            if a <= s < b:
                bucket[(short(n), g, bl)].append((s, e, qid))
        per_win.append(bucket)
    # node -> (key, occurrence index in topological order)
    occ = collections.Counter()
    nk = {}
    for i in order:
        nd = nodes[i]
        if not nd.get("name"):
            continue
        kk = key(nd["dname"], nd["grid"], nd["block"])
        nk[i] = (kk, occ[kk])
        occ[kk] += 1
    dur = {}
    miss = 0
    for i, (kk, o) in nk.items():
        ds = [(w[kk][o][1] - w[kk][o][0]) / 1e3 for w in per_win if len(w.get(kk, [])) > o]
        if ds:
            dur[i] = statistics.median(ds)
        else:
            miss += 1
            dur[i] = 0.0
    # longest path
    fin, best_pred = {}, {}
    for i in order:
        st = max((fin[p] for p in preds[i]), default=0.0)
        best_pred[i] = max(preds[i], key=lambda p: fin[p]) if preds[i] else None
        fin[i] = st + dur.get(i, 0.0)
    end = max(fin, key=fin.get)
    path = []
    while end is not None:
        path.append(end)
        end = best_pred[end]
    path.reverse()
    wl = [(b - a) / 1e3 for a, b in wins]
    print(f"nodes {len(nodes)} (kernels {len(nk)}, unmatched {miss}), edges {len(edges)}, windows {len(wins)}")
    print(f"measured replay window: median {statistics.median(wl):.1f} us" if wl else "no windows")
    print(f"longest dependency path: {fin[path[-1]]:.1f} us over {len(path)} nodes")
    for i in path:
        nd = nodes[i]
        print(f"  {fin[i] - dur.get(i, 0):8.1f} {dur.get(i, 0):7.1f}  {short(nd.get('dname') or nd['kind'])}")
    # late starts in the last full window
    if per_win:
        w = per_win[-2] if len(per_win) > 1 else per_win[-1]
        t0 = wins[-2][0] if len(per_win) > 1 else wins[-1][0]
        se = {}
        for i, (kk, o) in nk.items():
            if len(w.get(kk, [])) > o:
                se[i] = w[kk][o]
        late = []
        for i in se:
            pe = [se[p][1] for p in preds[i] if p in se]
            if pe:
                late.append(((se[i][0] - max(pe)) / 1e3, i))
        late.sort(reverse=True)
        print("largest late starts (start - latest predecessor end), last window:")
        for d, i in late[:25]:
            nd = nodes[i]
            print(f"  {d:7.1f} us  at {(se[i][0] - t0) / 1e3:8.1f}  q{se[i][2]}  {short(nd['dname'])}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
