"""Isolated timing of the small Cayley map kernels (k_small_cayley_fwd / _bwd) at the step's shapes:
the head's 512 -> 10 map (W [10][512], one workgroup) and the dynamics' three 128 x 10 maps (batch
3).  Run under rocprofv3 --kernel-trace for the kernels' own durations (the event times here include the
host's launch and autograd overhead).
(tools; not a test)

usage: python tools/probes/small_cayley_probe.py
"""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "fi-ode_amd"))
from fiode_amd.cayley import _SmallCayleyFn  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for name, shape in (("head_512x10", (1, 10, 512)), ("dyn_3x128x10", (3, 128, 10))):
    g = torch.Generator(device="cpu").manual_seed(0)
    W = torch.randn(*shape, generator=g).to(dev).requires_grad_(True)
    a = torch.rand(shape[0], generator=g).add(0.5).to(dev).requires_grad_(True)
    G = torch.randn(*shape, generator=g).to(dev)
    for _ in range(20):
        Q = _SmallCayleyFn.apply(W, a)
        Q.backward(G)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    n = 200
    e[0].record()
    for _ in range(n):
        Q = _SmallCayleyFn.apply(W, a)
    e[1].record()
    for _ in range(n):
        torch.autograd.grad(Q, (W, a), G, retain_graph=True)
    e[2].record()
    torch.cuda.synchronize()
    out[name] = {"fwd_us": round(e[0].elapsed_time(e[1]) / n * 1e3, 2),
                 "bwd_us_incl_glue": round(e[1].elapsed_time(e[2]) / n * 1e3, 2)}
print(json.dumps(out), flush=True)
