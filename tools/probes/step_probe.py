"""GPU-time decomposition of the configs[1] training step by hipGraph replays of its parts (not a
test): each part is captured alone and replayed, so the numbers carry no host dispatch cost.

python tools/probes/step_probe.py  ->  one JSON line of per-part ms
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def _cal():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    a.record()
    torch.cuda._sleep(1_000_000)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1_000_000          # ms per _sleep cycle


MS_PER_CYCLE = None


def graph_ms(fn, reps=5, warm=3):
    """GPU time of fn() dispatched eagerly behind a long _sleep (so the host runs ahead and the
    events see back-to-back GPU work, no dispatch gaps); the median of reps."""
    global MS_PER_CYCLE
    if MS_PER_CYCLE is None:
        MS_PER_CYCLE = _cal()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(60.0 / MS_PER_CYCLE))   # 60 ms head start for the host
        a.record()
        t0 = time.perf_counter()
        fn()
        host = (time.perf_counter() - t0) * 1e3
        b.record()
        torch.cuda.synchronize()
        assert host < 55.0, f"host enqueue {host:.1f} ms exceeds the head start"
        out.append(a.elapsed_time(b))
    ms = round(sorted(out)[len(out) // 2], 4)
    print(getattr(fn, "__name__", "?"), ms, f"host {host:.2f} ms", file=sys.stderr, flush=True)
    return ms


res = {}
print('start', file=sys.stderr, flush=True)
mod = bench.build_module(dev, train_ode=True)
x = torch.rand(128, 3, 32, 32, device=dev)
y = torch.randint(0, 10, (128,), device=dev)
bb = mod.init_coordinates.param_map
params = [p for p in bb.parameters() if p.requires_grad]
bb(x)          # sets each CayleyConv's input size and alpha

# 1. backbone fwd+bwd including its Cayley maps (serial, no side streams)
def bb_fb():
    for p in params:
        p.grad = None
    bb(x).sum().backward()
res["backbone_fwd_bwd_with_cayley"] = graph_ms(bb_fb)

# 2. the Cayley maps of the backbone alone (fwd + bwd)
from fiode_amd.cayley import CayleyConv, CayleyLinear  # noqa: E402
lays = [m for m in bb.modules() if isinstance(m, (CayleyConv, CayleyLinear))]
for m in lays:
    if isinstance(m, CayleyConv):
        assert m._n is not None


def cay_fb():
    for p in params:
        p.grad = None
    tot = 0.0
    for m in lays:
        Q = m.spectral_weight(m._n, dev) if isinstance(m, CayleyConv) else m.effective_weight()
        tot = tot + (Q.real.sum() if Q.is_complex() else Q.sum())
    tot.backward()
res["backbone_cayley_maps_fwd_bwd"] = graph_ms(cay_fb)
for i, m in enumerate(lays):
    def one(m=m):
        for p in params:
            p.grad = None
        Q = m.spectral_weight(m._n, dev) if isinstance(m, CayleyConv) else m.effective_weight()
        (Q.real.sum() if Q.is_complex() else Q.sum()).backward()
    res[f"cayley_{i}_{m.__class__.__name__}_{tuple(m.weight.shape)}"] = graph_ms(one)

# 3. backbone fwd+bwd with the maps frozen (convs, linears, GroupSort only)
frozen = {}
with torch.no_grad():
    for m in lays:
        frozen[m] = (m.spectral_weight(m._n, dev) if isinstance(m, CayleyConv) else m.effective_weight()).detach()
orig = {}
for m in lays:
    if isinstance(m, CayleyConv):
        orig[m] = m._take_spectral
        m._take_spectral = (lambda n, d, m=m: frozen[m])
    else:
        m._pre = None
        orig[m] = m.effective_weight
        m.effective_weight = (lambda m=m: frozen[m])
xr = x.clone().requires_grad_(True)


def bb_frozen():
    xr.grad = None
    bb(xr).sum().backward()
res["backbone_fwd_bwd_frozen_maps"] = graph_ms(bb_frozen)
with torch.no_grad():
    res["backbone_fwd_frozen_maps"] = graph_ms(lambda: bb(x))
for m in lays:
    if isinstance(m, CayleyConv):
        m._take_spectral = orig[m]
    else:
        m.effective_weight = orig[m]

# 4. dynamics Cayley maps fwd+bwd
dyn = mod.dyn_fun


def dyn_fb():
    w = dyn._effective_weights()
    sum(v.sum() for v in w.values()).backward()
res["dynamics_cayley_fwd_bwd"] = graph_ms(dyn_fb)

# 5. fused fan-out + train_ode kernels (ops level)
from fiode_amd import ops  # noqa: E402
with torch.no_grad():
    feat = bb(x).float().contiguous()
    w = {k: v.detach().float().contiguous() for k, v in dyn.effective_weights().items()}
plan = mod.step_plan(y)
res["lyap_step_kernels"] = graph_ms(lambda: ops.lyap_step(
    feat, y, w, plan["dyn"], sample_size=plan["S"], n_uniform=plan["S1"], sampler=plan["sampler"],
    dropout_mode=plan["dropout_mode"], kappa=plan["kappa"], seed=plan["seed"], offset=0))
oplan = mod.ode_plan(128)
h0 = torch.full((128, 10), 0.1, device=dev)


def ot():
    yo, _, ws = ops.odetrain_forward(feat, h0, w, oplan["dyn"], oplan["cfg"])
    ops.odetrain_backward(torch.ones_like(yo), feat, w, oplan["dyn"], oplan["cfg"], ws)
res["odetrain_fwd_bwd_kernels"] = graph_ms(ot)

# 6. Adam alone
opt = mod.configure_optimizers(capturable=True)[0][0]
for p in mod.parameters():
    p.grad = torch.zeros_like(p)
res["adam"] = graph_ms(lambda: opt.step())
print(json.dumps(res), flush=True)
