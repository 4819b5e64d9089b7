"""Forward / backward time of the dopri5 train_ode solve per eval (not a test): B = 128, random
weights and features, Philox dropout; prints NFE, attempts and us per eval for both kernels."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
for B in (128, 1024):
    P = make_params(seed=1)
    rng = np.random.default_rng(2)
    x = torch.from_numpy(rng.normal(size=(B, 10)).astype(np.float32)).to(dev)
    h0 = torch.full((B, 10), 0.1, device=dev)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
    for method, step in (("dopri5", 0.0), ("rk4", 0.1)):
        cfg = ops.odetrain_config(B, 0.0, 1.0, step, L.FIODE_DROPOUT_PHILOX, seed=3, offset=1, method=method,
                                  rtol=1e-3, atol=1e-3, max_attempts=64) if method == "dopri5" else \
            ops.odetrain_config(B, 0.0, 1.0, step, L.FIODE_DROPOUT_PHILOX, seed=3, offset=1)
        tf, tb = [], []
        for rep in range(4):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            y, st, ws = ops.odetrain_forward(x, h0, w, dyn, cfg)
            e1.record()
            ops.odetrain_backward(torch.ones_like(y), x, w, dyn, cfg, ws)
            e2.record()
            torch.cuda.synchronize()
            tf.append(e0.elapsed_time(e1) * 1e3)
            tb.append(e1.elapsed_time(e2) * 1e3)
        s = st.cpu().numpy()
        nfe = int(s[0])
        print(f"B={B} {method}: nfe {nfe} attempts {int(s[6]) if method == 'dopri5' else '-'}  fwd {min(tf):.0f} us "
              f"({min(tf) / nfe:.2f} us/eval)  bwd (+wgrad) {min(tb):.0f} us ({min(tb) / nfe:.2f} us/eval)", flush=True)
