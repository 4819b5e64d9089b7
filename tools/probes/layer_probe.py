"""Per-layer fwd / fwd+bwd GPU time of the backbone + dynamics Cayley maps (not a test)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
import bench
dev = torch.device("cuda:0")
mod = bench.build_module(dev)

def tm(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3

from torch.profiler import profile, ProfilerActivity
x = torch.rand(128, 3, 32, 32, device=dev)
bb = mod.init_coordinates.param_map
h = bb[0](x)
for i, m in enumerate(bb[1].model):
    hin = h.detach().requires_grad_(True)
    out = m(hin)
    g = torch.randn_like(out)
    f = tm(lambda: m(hin))
    def fb():
        o = m(hin)
        o.backward(g)
    fbt = tm(fb)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fb(); torch.cuda.synchronize()
    nk = sum(1 for e in prof.events() if e.device_type.name == "CUDA")
    print(f"{i:2d} {m.__class__.__name__:13s} {tuple(hin.shape)!s:22s} fwd {f:8.1f} us  fwd+bwd {fbt:8.1f} us  kernels {nk}", flush=True)
    h = out.detach()
dyn = mod.dyn_fun
def dfb():
    w = dyn.effective_weights()
    s = sum((v * v).sum() for v in w.values())
    s.backward()
print(f"dynamics Cayley maps fwd+bwd {tm(dfb):8.1f} us", flush=True)
