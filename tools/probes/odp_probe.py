"""Phase timing of the dopri5 train solve k_odp_fwd / k_odp_bwd at B=128 (the bench's configs[2]
dynamics: scale_nominal, dropout 0.5; needs tools/libfiode_prof.so, `make -C fi-ode_amd/csrc prof`;
not a test).  Block 0's wall-clock ticks per phase of every eval, against the rk4 solve."""
import os
import pathlib
import sys
import ctypes as ct

ROOT = pathlib.Path(__file__).resolve().parents[2]
os.environ.setdefault("FIODE_LIB", str(ROOT / "tools" / "libfiode_prof.so"))
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
dyn = ops.DynCfg(scale_nominal=True, dropout=0.5)
al = lambda v: (v + 255) & ~255
for method, A in (("rk4", 0), ("dopri5", 64), ("dopri5", ops.odetrain_default_attempts(B))):
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3, method=method,
                              max_attempts=max(A, 1))
    E = ops.odetrain_evals(cfg)
    for rep in range(3):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        y, st, ws = ops.odetrain_forward(x, h0, w, dyn, cfg)
        e1.record()
        torch.cuda.synchronize()
        offs = (ct.c_int64 * L.FIODE_ODETRAIN_NSAVED)()
        L.lib().fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(offs, ct.c_void_p))
        xs = offs[7] + al(B * E * 10 * 4)
        nt4 = (B + 3) // 4
        base = xs + (4 * 2 * nt4 * 16 + 8) * 8
        prof = ws[base: base + 16 * 8].view(torch.int64).cpu().numpy().astype(np.float64)
        ops.odetrain_backward(torch.ones_like(y), x, w, dyn, cfg, ws)
        e2.record()
        torch.cuda.synchronize()
        pb = ws[base: base + 16 * 8].view(torch.int64).cpu().numpy().astype(np.float64) - prof
    s = st.cpu().tolist()
    nfe = s[0]
    t = prof / max(nfe, 1) * 0.01          # us per eval
    fwd = e0.elapsed_time(e1) * 1e3
    print(f"{method} A={A} E={E}: NFE {nfe} (accepted {s[4]}, rejected {s[5]}), forward {fwd:.0f} us = "
          f"{fwd / max(nfe, 1):.2f} us/eval, backward {e1.elapsed_time(e2) * 1e3:.0f} us; per eval (block 0): "
          f"mlp {t[1]:.2f}  nominal {t[5]:.2f}  QP+exit {t[3]:.2f} (bisection {t[6]:.2f}, exchange wait {t[7]:.2f})  "
          f"finalize {t[4]:.2f}  -> in-eval {t[1] + t[5] + t[3] + t[4]:.2f}", flush=True)
    if method == "dopri5":
        na = max(s[6], 1)
        print(f"    per attempt ({na}): loop {prof[2] / na * 0.01:.2f} us, batch sums {prof[9] / na * 0.01:.2f} us "
              f"(all {prof[9] * 0.01:.1f} us), evals {(t[1] + t[5] + t[3] + t[4]) * nfe / na:.2f} us; keep-word fetch "
              f"{prof[10] / na * 0.01:.2f}, stage inputs {prof[11] / na * 0.01:.2f}, error {prof[12] / na * 0.01:.2f}, "
              f"controller {prof[13] / na * 0.01:.2f} us", flush=True)
        print(f"    backward per attempt: loop {pb[0] / na * 0.01:.2f} us, batch sums {pb[9] / na * 0.01:.2f} us, "
              f"VJP phases {pb[10:16].sum() / na * 0.01:.2f} us ({pb[10:16].sum() / max(nfe, 1) * 0.01:.2f} per VJP), "
              f"vjp calls {pb[1] / na * 0.01:.2f}, stage-term loops {pb[3] / na * 0.01:.2f}, error adjoint "
              f"{pb[4] / na * 0.01:.2f}, prologue {pb[5] / na * 0.01:.2f} us", flush=True)
