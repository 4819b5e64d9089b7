"""Layer-by-layer check of one train_ode eval of the forward against numpy (not a test):
saved stage input h, a1, a2, ftilde of eval e vs the MLP recomputed from h with the given masks."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
B, p = int(sys.argv[1]) if len(sys.argv) > 1 else 8, 0.5
P = make_params(seed=5)
rng = np.random.default_rng(12)
x = rng.normal(size=(B, 10)).astype(np.float32)
h0 = np.full((B, 10), 0.1, np.float32)
cfg = ops.odetrain_config(B, 0.0, 1.0, 0.25, L.FIODE_DROPOUT_GIVEN)
E = ops.odetrain_evals(cfg)
masks = (rng.random((E, 2, B, 128)) >= p).astype(np.uint8)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
dyn = ops.DynCfg(scale_nominal=False, dropout=p)
y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                 masks=torch.from_numpy(masks).to(dev))
torch.cuda.synchronize()
sv = {k: v.cpu().numpy() for k, v in ops.odetrain_saved(ws, cfg).items()}
u = x @ P.Qx.T + P.bx + P.b1
for e in (0, 1):
    h = sv["h"][:, e]
    z1 = u + h @ P.Q1.T
    a1 = np.where(masks[e, 0] > 0, np.maximum(z1 * 2.0, 0), 0)
    z2 = P.b2 + sv["a1"][:, e] @ P.Q2.T
    a2 = np.where(masks[e, 1] > 0, np.maximum(z2 * 2.0, 0), 0)
    ft = P.b3 + sv["a2"][:, e] @ P.Q3.T
    print(f"eval {e}: a1 err {np.abs(a1 - sv['a1'][:, e]).max():.3g}  a2 err {np.abs(a2 - sv['a2'][:, e]).max():.3g}  "
          f"ft err {np.abs(ft - sv['ftilde'][:, e]).max():.3g}  (scale {np.abs(ft).max():.3g})")
    if e == 0:
        d1 = np.abs(a1 - sv["a1"][:, e])
        bad = np.argwhere(d1 > 1e-4)
        print("  a1 bad (row, unit) first 12:", bad[:12].tolist())
        d2 = np.abs(a2 - sv["a2"][:, e])
        print("  a2 bad (row, unit) first 12:", np.argwhere(d2 > 1e-4)[:12].tolist())
        print("  ft dev:", np.round(sv["ftilde"][0, e], 4).tolist(), "\n  ft ref:", np.round(ft[0], 4).tolist())
