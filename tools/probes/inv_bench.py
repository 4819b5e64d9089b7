"""Micro-benchmark of fiode_batched_inverse (not a test)."""
import sys, pathlib, time
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
from fiode_amd import ops
from fiode_amd.cayley import _block_inverse
dev = torch.device("cuda:0")

def tm(fn, reps=50):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3

for dt in (torch.float32, torch.complex64):
    for n, bs in [(3, 544), (10, 1), (16, 1), (32, 1), (32, 144), (64, 1), (64, 40), (128, 1), (128, 8)]:
        M = torch.eye(n, dtype=dt, device=dev) + 0.1 * torch.randn(bs, n, n, dtype=dt, device=dev)
        out = torch.empty_like(M)
        print(dt, n, bs, f"{tm(lambda: ops.batched_inverse(M, out=out)):.1f} us", flush=True)
M = torch.eye(512, device=dev) + 0.01 * torch.randn(512, 512, device=dev)
print("block 512", f"{tm(lambda: _block_inverse(M)):.1f} us")
print("linalg.inv 512", f"{tm(lambda: torch.linalg.inv(M)):.1f} us")
