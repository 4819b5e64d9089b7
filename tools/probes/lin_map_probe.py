"""Latency of the backbone CayleyLinear maps, part by part, as hipGraph replays (not a test).

python tools/probes/lin_map_probe.py  ->  one JSON line of us per replay
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import ops  # noqa: E402
from fiode_amd.cayley import CayleyLinear  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def replay_us(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 2)


mod = bench.build_module(dev, train_ode=True)
lins = [m for m in mod.init_coordinates.modules() if isinstance(m, CayleyLinear)]
res = {}
for m in lins:
    name = f"lin{m.weight.shape[1]}x{m.weight.shape[0]}"
    W = m.weight

    def fwd():
        with torch.no_grad():
            m.effective_weight()

    def fwdbwd():
        Q = m.effective_weight()
        Q.backward(torch.ones_like(Q))

    res[name + "_fwd"] = replay_us(fwd)
    res[name + "_fwdbwd"] = replay_us(fwdbwd)
    for p in m.parameters():
        p.grad = None

for n in (512, 128):
    A = torch.randn(n, n, device=dev) * 0.05
    M = torch.eye(n, device=dev) + (A - A.T) + A.T @ A
    res[f"block_inverse{n}"] = replay_us(lambda: ops.block_inverse(M))
    try:
        res[f"torch_inv{n}"] = replay_us(lambda: torch.linalg.inv(M))
    except Exception as e:  # noqa: BLE001
        res[f"torch_inv{n}"] = f"failed {str(e)[:60]}"
Vp = torch.randn(3584, 512, device=dev)
res["gemm_512x3584x512"] = replay_us(lambda: torch.matmul(Vp.mT, Vp))
X = torch.randn(512, 512, device=dev)
res["gemm_512^3"] = replay_us(lambda: torch.matmul(X, X))
print(json.dumps(res), flush=True)
