"""Node-by-node listing of the step DAG (tools/probes/graph_dag_probe.py) with the queue, start and
duration each node had in the last replay of a kernel trace (approximate occurrence matching).
usage: python tools/dag_nodes.py <step.dot> <run_kernel_trace.csv>  (tools; not a test)"""
import sys, collections, statistics
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import dag_critical as D
import re, csv
dot, trace = sys.argv[1], sys.argv[2]
txt=open(dot).read()
nodes={}
for m in re.finditer(r'"graph_\d+_node_(\d+)"\[style="\w+"shape="record"label="\{\n(\w+)\n(.*?)\}"\];', txt, re.S):
    nid, kind, body = int(m.group(1)), m.group(2), m.group(3)
    k = re.search(r"\{ID \| \d+ \| (.*?)\\<\\<\\<\((\d+),(\d+),(\d+)\),\((\d+),(\d+),(\d+)\)", body)
    nodes[nid]={"kind":kind,"name":k.group(1) if k else kind,"grid":tuple(int(k.group(i)) for i in (2,3,4)) if k else None,"block":tuple(int(k.group(i)) for i in (5,6,7)) if k else None}
edges=[(int(a),int(b)) for a,b in re.findall(r'"graph_\d+_node_(\d+)" -> "graph_\d+_node_(\d+)"', txt)]
names=[nodes[i]["name"] for i in sorted(nodes)]
dem=D.demangle(names)
for i,d in zip(sorted(nodes),dem): nodes[i]["d"]=D.short(d)
preds=collections.defaultdict(list); succ=collections.defaultdict(list)
for a,b in edges: preds[b].append(a); succ[a].append(b)
rows=list(csv.DictReader(open(trace)))
ks=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),D.short(r["Kernel_Name"]),(int(r["Grid_Size_X"]),int(r["Grid_Size_Y"]),int(r["Grid_Size_Z"])),r["Queue_Id"]) for r in rows)
# take the last 1 replay: kernels after the last graph-root occurrence... use last 152 kernel launches
last=ks[-150:]
t0=last[0][0]
byk=collections.defaultdict(list)
for s,e,n,g,q in last: byk[(n,g)].append((s,e,q))
occ=collections.Counter()
for i in sorted(nodes):
    nd=nodes[i]
    if nd["grid"] is None:
        print(f"{i:4d} {nd['kind']:8s} preds {preds[i]} succ {succ[i]}"); continue
    key=(nd["d"], tuple(a*b for a,b in zip(nd["grid"],nd["block"])))
    o=occ[key]; occ[key]+=1
    L=byk.get(key,[])
    s,e,q = L[o] if o<len(L) else (0,0,'?')
    print(f"{i:4d} q{q} {(s-t0)/1e3:8.1f} {(e-s)/1e3:6.1f} {nd['d'][:40]:40s} preds {preds[i]} succ {succ[i]}")
