"""What sits on the critical path of the replayed configs[1] step (not a test): the hipGraph step
time with parts of the work frozen (their outputs precomputed, their backward dropped).  The
differences against the full step bound each part's exposed (non-overlapped) time.

python tools/probes/critical_probe.py  ->  one JSON line of ms per step per variant
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.cayley import CayleyConv, CayleyLinear  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def step_ms(mod, steps=30):
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    gs = GraphTrainStep(mod, opt, x, y)
    for _ in range(5):
        gs.step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        gs.step()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / steps * 1e3, 4)


def freeze(mod, convs=False, linears=False, dyn=False):
    x = torch.rand(128, 3, 32, 32, device=dev)
    mod.init_coordinates.param_map(x)            # conv input sizes, alpha init
    for m in mod.init_coordinates.modules():
        if convs and isinstance(m, CayleyConv):
            Q = m.spectral_weight(m._n, dev).detach()
            m.spectral_weight = (lambda n, d, Q=Q: Q)
            m.prefetch = (lambda s: None)
        if linears and isinstance(m, CayleyLinear):
            Q = m.effective_weight().detach()
            m.effective_weight = (lambda Q=Q: Q)
            m.prefetch = (lambda s: None)
    if dyn:
        w = {k: v.detach() for k, v in mod.dyn_fun._effective_weights().items()}
        mod.dyn_fun._effective_weights = (lambda w=w: w)
        mod.dyn_fun.prefetch = (lambda s: None)     # nothing to overlap (a side-stream no-op is unjoined work)


res = {}
for name, kw, ode in [("frozen_linear_maps", dict(linears=True), True), ("frozen_dyn_maps", dict(dyn=True), True),
                      ("frozen_lin_dyn_maps", dict(linears=True, dyn=True), True),
                      ("frozen_lin_dyn_maps_lyap_only", dict(linears=True, dyn=True), False),
                      ("frozen_conv_maps", dict(convs=True), True)]:
    mod = bench.build_module(dev, train_ode=ode)
    if kw:
        freeze(mod, **kw)
    try:
        res[name] = step_ms(mod)
    except Exception as e:          # noqa: BLE001 - a variant that cannot be captured is reported
        res[name] = f"failed: {str(e).splitlines()[0][:80]}"
        torch.cuda.synchronize()
    print(name, res[name], file=sys.stderr, flush=True)
print(json.dumps(res), flush=True)
