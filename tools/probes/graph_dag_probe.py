"""Export the captured configs[1] training step's hipGraph -- its nodes (kernel names, grid sizes)
and dependency edges -- as JSON, and replay it a few times, so that tools/dag_critical.py can put the
kernels' measured durations (run this under rocprofv3 --kernel-trace) on the DAG and find the longest
dependency path.  (tools; not a test)

usage: python tools/probes/graph_dag_probe.py <out_dir> [replays]
"""
import ctypes as ct
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fi-ode_amd"))
import bench  # noqa: E402
from fiode_amd import graph_step as GS  # noqa: E402

out = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
os.makedirs(out, exist_ok=True)


class _KeepGraph(torch.cuda.CUDAGraph):
    def __new__(cls, keep_graph=False):
        return super().__new__(cls, True)

    def __init__(self, keep_graph=False):
        super().__init__(True)


GS.torch.cuda.CUDAGraph = _KeepGraph           # graph_step's captures keep their hipGraph_t
dev = torch.device("cuda:0")
mod = bench.build_module(dev, train_ode=True)
if os.environ.get("FIODE_PROBE_LATE_AT") is not None:     # the map-prefetch split point (None: all first)
    v = os.environ["FIODE_PROBE_LATE_AT"]
    mod._prefetch_late_at = None if v == "none" else int(v)
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
gs = GS.GraphTrainStep(mod, opt, x, y, placement_trials=int(os.environ.get("FIODE_PLACEMENT_TRIALS", "1")))
raw = gs.g_fb.raw_cuda_graph()

hip = ct.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
vp = ct.c_void_p
hip.hipGraphGetNodes.argtypes = [vp, ct.POINTER(vp), ct.POINTER(ct.c_size_t)]
hip.hipGraphGetEdges.argtypes = [vp, ct.POINTER(vp), ct.POINTER(vp), ct.POINTER(ct.c_size_t)]
hip.hipGraphNodeGetType.argtypes = [vp, ct.POINTER(ct.c_int)]
hip.hipKernelNameRefByPtr.argtypes = [vp, vp]
hip.hipKernelNameRefByPtr.restype = ct.c_char_p
hip.hipGraphDebugDotPrint.argtypes = [vp, ct.c_char_p, ct.c_uint]


class Dim3(ct.Structure):
    _fields_ = [("x", ct.c_uint32), ("y", ct.c_uint32), ("z", ct.c_uint32)]


class KParams(ct.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", vp), ("func", vp), ("gridDim", Dim3), ("kernelParams", vp),
                ("sharedMemBytes", ct.c_uint)]


hip.hipGraphKernelNodeGetParams.argtypes = [vp, ct.POINTER(KParams)]
rc_dot = hip.hipGraphDebugDotPrint(vp(raw), os.path.join(out, "step.dot").encode(), 1 << 0)

n = ct.c_size_t(0)
assert hip.hipGraphGetNodes(vp(raw), None, ct.byref(n)) == 0
nodes = (vp * n.value)()
assert hip.hipGraphGetNodes(vp(raw), nodes, ct.byref(n)) == 0
idx = {nodes[i]: i for i in range(n.value)}
info = []
for i in range(n.value):
    t = ct.c_int(-1)
    hip.hipGraphNodeGetType(vp(nodes[i]), ct.byref(t))
    d = {"type": t.value}
    if t.value == 0:                       # hipGraphNodeTypeKernel
        p = KParams()
        if hip.hipGraphKernelNodeGetParams(vp(nodes[i]), ct.byref(p)) == 0:
            name = hip.hipKernelNameRefByPtr(vp(p.func), None) if p.func else None
            d.update(name=(name or b"?").decode(errors="replace"), grid=[p.gridDim.x, p.gridDim.y, p.gridDim.z],
                     block=[p.blockDim.x, p.blockDim.y, p.blockDim.z])
    info.append(d)
m = ct.c_size_t(0)
assert hip.hipGraphGetEdges(vp(raw), None, None, ct.byref(m)) == 0
fr, to = (vp * m.value)(), (vp * m.value)()
assert hip.hipGraphGetEdges(vp(raw), fr, to, ct.byref(m)) == 0
edges = [[idx[fr[i]], idx[to[i]]] for i in range(m.value)]
json.dump({"nodes": info, "edges": edges, "dot_rc": rc_dot}, open(os.path.join(out, "step_dag.json"), "w"))
print(f"nodes {n.value} edges {m.value} dot rc {rc_dot}", flush=True)
for _ in range(reps):
    gs.step()
torch.cuda.synchronize()
gs.close()
