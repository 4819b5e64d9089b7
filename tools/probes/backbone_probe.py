"""Timing probe: where does the backbone's time go (not a test)."""
import sys, time, pathlib, json
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
dev = torch.device("cuda:0")

def tm(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3

res = {}
for lib in ("default", "magma", "cusolver"):
    try:
        torch.backends.cuda.preferred_linalg_library(lib)
    except Exception as e:
        res[lib] = str(e); continue
    r = {}
    for shape, dt in [((544, 3, 3), torch.complex64), ((144, 32, 32), torch.complex64), ((40, 64, 64), torch.complex64),
                      ((512, 512), torch.float32), ((10, 10), torch.float32), ((128, 128), torch.float32)]:
        M = torch.eye(shape[-1], dtype=dt, device=dev) + 0.1 * torch.randn(shape, dtype=dt, device=dev)
        try:
            r[f"inv{shape}"] = round(tm(lambda: torch.linalg.inv(M)), 4)
            r[f"inv_ex{shape}"] = round(tm(lambda: torch.linalg.inv_ex(M)[0]), 4)
        except Exception as e:
            r[f"inv{shape}"] = str(e)[:80]
    res[lib] = r
torch.backends.cuda.preferred_linalg_library("default")
print(json.dumps(res, indent=1), flush=True)

import bench
mod = bench.build_module(dev)
x = torch.rand(128, 3, 32, 32, device=dev)
bb = mod.init_coordinates.param_map
def fb():
    out = bb(x)
    out.sum().backward()
print("backbone fwd+bwd ms", tm(fb), flush=True)
print("backbone fwd ms", tm(lambda: bb(x)), flush=True)
for i, m in enumerate(bb[1].model):
    if hasattr(m, "effective_weight") or m.__class__.__name__ == "CayleyConv":
        pass
# per-layer forward timing
h = bb[0](x)
for i, m in enumerate(bb[1].model):
    t = tm(lambda: m(h), reps=10)
    print(i, m.__class__.__name__, tuple(h.shape), f"{t:.3f} ms", flush=True)
    h = m(h).detach()
y = torch.randint(0, 10, (128,), device=dev)
opt = mod.configure_optimizers()[0][0]
def step():
    opt.zero_grad()
    loss = mod.compute_loss(x, y, 128, "relu")
    loss.backward()
    opt.step()
print("full step ms", tm(step), flush=True)
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(3):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40), flush=True)
