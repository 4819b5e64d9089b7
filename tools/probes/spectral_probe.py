"""Per-kernel view of the fused spectral Cayley maps of the four KWLarge convs (not a test):
run under rocprofv3 --kernel-trace --stats."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

from fiode_amd.cayley import CayleyConv  # noqa: E402

dev = torch.device("cuda:0")
layers = []
for cout, cin, n in [(32, 3, 32), (32, 128, 16), (64, 32, 16), (64, 256, 8)]:
    c = CayleyConv(cin, cout, 3).to(dev)
    c.spectral_weight(n, dev)          # alpha init
    layers.append((c, n))
for rep in range(10):
    for c, n in layers:
        Q = c.spectral_weight(n, dev)
        Q.backward(torch.ones_like(Q))
torch.cuda.synchronize()
print("ok")
