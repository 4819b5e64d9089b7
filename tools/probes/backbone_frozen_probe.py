"""Kernel composition of the backbone forward + backward with its Cayley maps frozen (not a test):
run under rocprofv3 --kernel-trace --stats; 20 iterations."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.cayley import CayleyConv, CayleyLinear  # noqa: E402

dev = torch.device("cuda:0")
mod = bench.build_module(dev, train_ode=True)
bb = mod.init_coordinates.param_map
x = torch.rand(128, 3, 32, 32, device=dev)
bb(x)
for m in bb.modules():
    if isinstance(m, CayleyConv):
        Q = m.spectral_weight(m._n, dev).detach()
        m._take_spectral = (lambda n, d, Q=Q: Q)
    elif isinstance(m, CayleyLinear):
        Q = m.effective_weight().detach()
        m.effective_weight = (lambda Q=Q: Q)
xr = x.clone().requires_grad_(True)
for _ in range(20):
    xr.grad = None
    bb(xr).sum().backward()
torch.cuda.synchronize()
print("ok")

if len(sys.argv) > 1 and sys.argv[1] == "ops":
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        for _ in range(5):
            xr.grad = None
            bb(xr).sum().backward()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=45, max_name_column_width=60), flush=True)
    ka = prof.key_averages(group_by_input_shape=True)
    rows = sorted([e for e in ka if e.key in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::_fft_r2c",
                                               "aten::_fft_c2r", "aten::_fft_c2c")],
                  key=lambda e: -e.self_device_time_total)
    for e in rows[:30]:
        print(f"{e.key:18s} n={e.count:4d} self_cuda={e.self_device_time_total / 5:8.1f}us/iter  shapes={str(e.input_shapes)[:150]}")
    ks = prof.key_averages(group_by_stack_n=6)
    rows = sorted([e for e in ks if e.key == "aten::copy_"], key=lambda e: -e.self_device_time_total)
    for e in rows[:12]:
        print(f"copy_ self_cuda={e.self_device_time_total / 5:8.1f}us/iter n={e.count}")
        for fr in (e.stack or [])[:6]:
            print("      ", fr)
