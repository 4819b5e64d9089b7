"""Probe (not a test): spectral Cayley map forward / backward time per KWLarge conv layer shape
(fiode_spectral_cayley_forward / _backward, 20 calls back to back between two events) and the
one-launch block inverse (n = 128, 512), for the library FIODE_LIB selects.

FIODE_LIB=... python tools/probes/spec_probe.py"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

from fiode_amd import ops, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


print("lib", L.LIB_PATH)
for (cout, cin, n) in [(32, 3, 32), (32, 128, 16), (64, 32, 16), (64, 256, 8)]:
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.1).to(dev)
    a = torch.ones(1, device=dev) * float(w.norm()) * 3.0
    Q, inv, ws = ops.spectral_cayley_forward(w, a, n)
    gQ = torch.randn(Q.shape, dtype=torch.complex64, generator=g).to(dev)
    tf = timed(lambda: ops.spectral_cayley_forward(w, a, n, out=(Q, inv, ws)))
    tb = timed(lambda: ops.spectral_cayley_backward(gQ, w, a, n, inv, ws))
    print(f"conv {cout}x{cin} n={n}: fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)
for n in (128, 512):
    A = torch.randn(n, n, generator=g, dtype=torch.float64) / n ** 0.5
    M = (torch.eye(n, dtype=torch.float64) + (A - A.T) + 0.3 * A.T @ A).float().to(dev)
    out = torch.empty_like(M)
    print(f"block inverse n={n}: {timed(lambda: ops.block_inverse(M, out=out)):7.1f} us", flush=True)
