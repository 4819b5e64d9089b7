"""k_lyap_wgrad phase stamps, cold vs warm operands (needs tools/libfiode_prof.so; not a test): the
train_ode solve at B=128 (rk4, 40 evals), the adjoint sweep, then the weight-gradient chain twice on
the same workspace -- the first right after the sweep wrote its operands, the second re-reading them."""
import ctypes as ct
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
os.environ["FIODE_LIB"] = str(ROOT / "tools" / "libfiode_prof.so")
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
B = 128
g = torch.Generator().manual_seed(0)
x = torch.randn(B, ops.X, generator=g).to(dev)
h0 = torch.full((B, 10), 0.1, device=dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3)
lib = L.lib()
lib.fiode_debug_wgrad_stamps.argtypes = [ct.c_void_p, ct.c_int]


def stamps():
    buf = (ct.c_ulonglong * 4096)()
    assert lib.fiode_debug_wgrad_stamps(buf, 4096) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4).astype(np.float64) * 0.01
    return st[st[:, 3] > 0]


def show(tag, st):
    t0 = st[:, 0].min()
    parts = ", ".join(f"{n} {np.median(st[:, k] - st[:, k - 1]):.2f}" for k, n in ((1, "stage"), (2, "mfma"), (3, "store")))
    print(f"{tag}: {len(st)} WGs, span {st[:, 3].max() - t0:.2f} us, p50 per phase: {parts}", flush=True)


for rep in range(3):
    y, stats, ws = ops.odetrain_forward(x, h0, w, dyn, cfg)
    gx = ops.odetrain_backward_x(torch.randn(B, 10, device=dev), x, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    ops.odetrain_backward_weights(x, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    show(f"rep {rep} after the sweep", stamps())
    ops.odetrain_backward_weights(x, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    show(f"rep {rep} re-run        ", stamps())
