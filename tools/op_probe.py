"""List the device kernels (with their aten op) of one conv / linear layer fwd+bwd (not a test)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
from torch.profiler import profile, ProfilerActivity
import bench
dev = torch.device("cuda:0")
mod = bench.build_module(dev)
bb = mod.init_coordinates.param_map[1].model
x = torch.rand(128, 32, 32, 32, device=dev)
for name, m, inp in (("conv2 (stride 2)", bb[2], x), ("linear 4096", bb[9], torch.rand(128, 4096, device=dev))):
    hin = inp.detach().requires_grad_(True)
    o = m(hin); o.backward(torch.randn_like(o)); torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        o = m(hin)
        o.backward(torch.randn_like(o))
        torch.cuda.synchronize()
    print(f"== {name}", flush=True)
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=45), flush=True)
