"""Device kernels by aten op for one backbone fwd+bwd (not a test)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
from torch.profiler import profile, ProfilerActivity
import bench
dev = torch.device("cuda:0")
mod = bench.build_module(dev)
bb = mod.init_coordinates.param_map
x = torch.rand(128, 3, 32, 32, device=dev)
for _ in range(2):
    o = bb(x); o.square().sum().backward()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    o = bb(x)
    o.square().sum().backward()
    torch.cuda.synchronize()
ka = prof.key_averages()
rows = sorted([e for e in ka if e.device_type.name == "CPU" and e.key.startswith("aten::")],
              key=lambda e: -e.device_time_total)
print(f"{'op':40s} {'calls':>6s} {'dev us':>9s}")
for e in rows[:40]:
    print(f"{e.key:40s} {e.count:6d} {e.device_time_total:9.1f}")
n_k = sum(e.count for e in ka if e.device_type.name == "CUDA")
print("device kernels:", n_k, " device time:", sum(e.self_device_time_total for e in ka if e.device_type.name == "CUDA"))

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof2:
    o = bb(x)
    o.square().sum().backward()
    torch.cuda.synchronize()
from collections import defaultdict
agg = defaultdict(lambda: [0, 0.0])
for e in prof2.events():
    if e.name in ("aten::clone", "aten::copy_") and e.device_type.name == "CPU":
        st = [f for f in (e.stack or []) if "fiode_amd" in f or "torch/fft" in f or "autograd" in f]
        key = (e.name, st[0] if st else "(autograd engine / c++)", str(e.input_shapes[:1]))
        agg[key][0] += 1
        agg[key][1] += e.device_time_total
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{c:4d} {t:8.1f}us  {k[0]:12s} {k[2][:40]:40s} {k[1][-90:]}")
