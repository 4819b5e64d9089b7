"""Event timing of the train_ode forward solves (not a test): rk4 at B = 128 (k_ot_fwd4) and
B = 2048 (16-row k_ot_fwd), dopri5 at B = 128 with the bench's configs[2] dynamics (k_odp_fwd).
Run once per library (FIODE_LIB) and compare the medians."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
for method, B, sn in (("rk4", 128, False), ("rk4", 2048, False), ("dopri5", 128, True)):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, ops.X, generator=g).to(dev)
    h0 = torch.full((B, 10), 0.1, device=dev)
    dyn = ops.DynCfg(scale_nominal=sn, dropout=0.5)
    kw = {} if method == "rk4" else {"method": "dopri5", "max_attempts": ops.odetrain_default_attempts(B)}
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3, **kw)
    ts, tb = [], []
    gy = torch.ones(B, 10, device=dev)
    for rep in range(25):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        y, st, ws = ops.odetrain_forward(x, h0, w, dyn, cfg)
        e1.record()
        grads, _ = ops.odetrain_backward(gy, x, w, dyn, cfg, ws)
        e2.record()
        torch.cuda.synchronize()
        if rep >= 5:
            ts.append(e0.elapsed_time(e1) * 1e3)
            tb.append(e1.elapsed_time(e2) * 1e3)
    stv = st.cpu().numpy().tolist()
    print(f"{method} B={B}: forward median {np.median(ts):.1f} us (min {min(ts):.1f}), backward median "
          f"{np.median(tb):.1f} us  stats {stv}  y sum {float(y.double().sum()):.9e}", flush=True)
