"""A few fused fan-out steps at the bench shape, for rocprofv3 --pmc passes (not a test)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np, torch
from fiode_amd import ops
from tests._util import make_params
dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
B, S = 128, 256
feat = torch.randn(B, 10, device=dev); y = torch.randint(0, 10, (B,), device=dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
for r in range(4):
    ops.lyap_step(feat, y, w, dyn, sample_size=S, n_uniform=204, offset=r)
torch.cuda.synchronize()
print("ok")
