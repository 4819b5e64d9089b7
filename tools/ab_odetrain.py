"""A/B bit-identity check of the train_ode solve between two builds of libfiode (not a test):
FIODE_LIB=<lib> python tools/ab_odetrain.py out.pt  writes y(t1) and the saved (mu, v, h) of a
seeded solve; compare two outputs with  python tools/ab_odetrain.py --cmp a.pt b.pt."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

if sys.argv[1] == "--cmp":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        print(k, "identical" if torch.equal(a[k], b[k]) else f"DIFFER max {float((a[k] - b[k]).abs().max())}")
    sys.exit(0 if all(torch.equal(a[k], b[k]) for k in a) else 1)

import numpy as np  # noqa: E402
from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for B, sn in ((128, False), (300, True), (37, False)):
    P = make_params(seed=B)
    rng = np.random.default_rng(B)
    x = torch.from_numpy(rng.normal(size=(B, 10)).astype(np.float32)).to(dev)
    h0 = torch.full((B, 10), 0.1, device=dev)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3, offset=5)
    y, st, ws = ops.odetrain_forward(x, h0, w, ops.DynCfg(scale_nominal=sn), cfg)
    sv = ops.odetrain_saved(ws, cfg)
    out.update({f"y{B}": y.cpu(), f"mu{B}": sv["mu"].cpu(), f"v{B}": sv["v"].cpu(), f"stats{B}": st.cpu()})
    gy = torch.from_numpy(rng.normal(size=(B, 10)).astype(np.float32)).to(dev)
    grads, _ = ops.odetrain_backward(gy, x, w, ops.DynCfg(scale_nominal=sn), cfg, ws)
    out.update({f"g{k}{B}": v.cpu() for k, v in grads.items()})
# the dopri5 train solve (bench configs[2] dynamics: scale_nominal, Philox dropout p = 0.5)
for B in (128, 300):
    P = make_params(seed=B + 1)
    rng = np.random.default_rng(B + 1)
    x = torch.from_numpy(rng.normal(size=(B, 10)).astype(np.float32)).to(dev)
    h0 = torch.full((B, 10), 0.1, device=dev)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    dyn = ops.DynCfg(scale_nominal=True, dropout=0.5)
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=5, offset=7, method="dopri5",
                              max_attempts=ops.odetrain_default_attempts(B))
    y, st, ws = ops.odetrain_forward(x, h0, w, dyn, cfg)
    out.update({f"dp_y{B}": y.cpu(), f"dp_stats{B}": st.cpu()})
    gy = torch.from_numpy(rng.normal(size=(B, 10)).astype(np.float32)).to(dev)
    grads, _ = ops.odetrain_backward(gy, x, w, dyn, cfg, ws)
    out.update({f"dp_g{k}{B}": v.cpu() for k, v in grads.items()})
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
