"""Dump the captured training step's hipGraph structure (not a test): the bench's configs[1] module
under GraphTrainStep, every CUDAGraph kept (keep_graph), then through the HIP graph API (ctypes):
each node's type and kernel name, and the edges -> gpurun_out/graph_dot/g<i>.json.  Read with
tools/probes/graph_dot_read.py: which graph edges a kernel waits on (e.g. the head's first backward
GEMM after k_ot_gx)."""
import ctypes
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

OUT = ROOT / "gpurun_out" / "graph_dot"
OUT.mkdir(parents=True, exist_ok=True)
_made = []
_Orig = torch.cuda.CUDAGraph


class _KeptGraph(_Orig):
    def __new__(cls, *a, **k):
        g = _Orig.__new__(cls, True)
        _made.append(g)
        return g

    def __init__(self, *a, **k):
        torch._C._CUDAGraph.__init__(self, True)


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KParams(ctypes.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p),
                ("gridDim", Dim3), ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


def dump(graph_ptr: int, path: pathlib.Path):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
    hip.hipKernelNameRefByPtr.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipKernelNameRef.restype = ctypes.c_char_p
    hip.hipKernelNameRef.argtypes = [ctypes.c_void_p]
    g = ctypes.c_void_p(graph_ptr)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    idx = {nodes[i]: i for i in range(n.value)}
    out = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        rec = {"i": i, "type": t.value}
        if t.value == 0:
            kp = KParams()
            if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nodes[i]), ctypes.byref(kp)) == 0 and kp.func:
                nm = hip.hipKernelNameRefByPtr(ctypes.c_void_p(kp.func), None)
                if not nm:
                    nm = hip.hipKernelNameRef(ctypes.c_void_p(kp.func))
                rec["name"] = nm.decode(errors="replace") if nm else None
                rec["grid"] = [kp.gridDim.x, kp.gridDim.y, kp.gridDim.z]
                rec["block"] = [kp.blockDim.x, kp.blockDim.y, kp.blockDim.z]
        out.append(rec)
    m = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(m)) == 0
    fr = (ctypes.c_void_p * m.value)()
    to = (ctypes.c_void_p * m.value)()
    assert hip.hipGraphGetEdges(g, fr, to, ctypes.byref(m)) == 0
    edges = [[idx[fr[k]], idx[to[k]]] for k in range(m.value)]
    path.write_text(json.dumps({"nodes": out, "edges": edges}))
    print("dumped", path, len(out), "nodes", len(edges), "edges", flush=True)


torch.cuda.CUDAGraph = _KeptGraph
dev = torch.device("cuda:0")
mod = bench.build_module(dev, seed=0, train_ode=True)
opt = mod.configure_optimizers(capturable=True)[0][0]
gen = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=gen).to(dev)
y = torch.randint(0, 10, (128,), generator=gen).to(dev)
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 4
replays = int(sys.argv[2]) if len(sys.argv) > 2 else 0
gs = GraphTrainStep(mod, opt, x, y, placement_trials=trials)
gs.step()
torch.cuda.synchronize()
print("placement", getattr(gs, "placement_ms", None), getattr(gs, "placement_pick", None), flush=True)
try:
    dump(gs.g_fb.raw_cuda_graph(), OUT / "step.json")
except Exception as e:  # noqa: BLE001
    print("dump failed", repr(e), flush=True)
for _ in range(replays):            # for a rocprofv3 kernel trace of the same graph
    gs.step()
torch.cuda.synchronize()
gs.close()
