"""Timings of BASELINE configs 3-5 on one MI355X (not a test): dopri5 validation solve, the T=40
certification grid, the large-batch fan-out step."""
import sys, pathlib, time, json
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np, torch
from fiode_amd import ops, _lib as L
from tests._util import make_params
dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
out = {}

def ev():
    return torch.cuda.Event(enable_timing=True)

# config 3: dopri5 tol 1e-3 validation solve, B=128 (and 4096)
for B in (128, 1024, 4096, 8192):
    x = torch.randn(B, 10, device=dev); h0 = torch.full((B, 10), 0.1, device=dev)
    times = torch.tensor([0.0, 1.0], dtype=torch.float64, device=dev)
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.0)
    for _ in range(2):
        ops.odeint_dyn(x, h0, times, w, dyn, method="dopri5", rtol=1e-3, atol=1e-3)
    a, b = ev(), ev(); a.record()
    sol, st, dst = ops.odeint_dyn(x, h0, times, w, dyn, method="dopri5", rtol=1e-3, atol=1e-3)
    b.record(); torch.cuda.synchronize()
    s = st.cpu().tolist()
    out[f"dopri5_B{B}"] = {"ms": round(a.elapsed_time(b), 3), "nfe": s[0], "accepted": s[1], "rejected": s[2], "status": s[3], "workgroups": s[6], "tiles_per_wg": s[7]}
    print(out[f"dopri5_B{B}"], flush=True)

# config 4: certification of one image on the T=40 grid (G = 41,320,837 rows)
grid = ops.certify_grid(40, device=dev)
torch.cuda.synchronize()
xf = torch.randn(10, device=dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.0)
ops.certify_image(xf, 3, grid, w, dyn, T=40, batches=10)
torch.cuda.synchronize()
a, b = ev(), ev(); a.record()
for lab in range(3):
    o, it = ops.certify_image(xf, lab, grid, w, dyn, T=40, batches=10)
b.record(); torch.cuda.synchronize()
ms = a.elapsed_time(b) / 3
G = grid.shape[0]
tf = 2 * 37888 * G / (ms * 1e-3) / 1e12    # pass-1 MLP FLOP (the QP pass reuses the MLP output)
out["certify_T40"] = {"ms_per_image": round(ms, 2), "rows": G, "rows_per_s": round(G / (ms * 1e-3) / 1e9, 2),
                      "note": "rows/s in 1e9; MLP once per row"}
print(out["certify_T40"], flush=True)

# config 5: the fused fan-out at B=1024 x S=1024 (one rank's rows)
B, S = 1024, 1024
feat = torch.randn(B, 10, device=dev); y = torch.randint(0, 10, (B,), device=dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
for r in range(2):
    ops.lyap_step(feat, y, w, dyn, sample_size=S, n_uniform=S * 4 // 5, offset=r)
torch.cuda.synchronize()
a, b = ev(), ev(); a.record()
for r in range(3):
    sc, g, _ = ops.lyap_step(feat, y, w, dyn, sample_size=S, n_uniform=S * 4 // 5, offset=10 + r)
b.record(); torch.cuda.synchronize()
ms = a.elapsed_time(b) / 3
out["fanout_B1024_S1024"] = {"ms": round(ms, 3), "rows": B * S,
                             "tflops": round(148992 * B * S / (ms * 1e-3) / 1e12, 2),
                             "loss": float(sc[0]), "finite": bool(all(torch.isfinite(v).all() for v in g.values()))}
print(out["fanout_B1024_S1024"], flush=True)
print(json.dumps(out))
