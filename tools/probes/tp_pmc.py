"""The throughput kernels once each, for rocprofv3 --pmc passes (not a test): 3 fused fan-out
steps at the bench shape (k_lyap_fwd / k_lyap_bwd), one at configs[4]'s B=1024 x S=1024 (the
dispatches with the larger grid) and one certification image on the T=40 grid (k_cert_fwd /
k_cert_final)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
B, S = 128, 256
g = torch.Generator().manual_seed(0)
feat = torch.randn(B, 10, generator=g).to(dev)
y = torch.randint(0, 10, (B,), generator=g).to(dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
for r in range(3):
    ops.lyap_step(feat, y, w, dyn, sample_size=S, n_uniform=204, offset=r)
fl = torch.randn(1024, 10, generator=g).to(dev)
yl = torch.randint(0, 10, (1024,), generator=g).to(dev)
ops.lyap_step(fl, yl, w, dyn, sample_size=1024, n_uniform=816, offset=7)
grid = ops.certify_grid(40, device=dev)
ops.certify_image(torch.randn(10, generator=g).to(dev), 3, grid, w, ops.DynCfg(scale_nominal=False, dropout=0.0),
                  T=40, batches=10)
torch.cuda.synchronize()
print("ok")
