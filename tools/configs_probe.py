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
# config 5 as a whole training step: B=1024 images x S=1024 samples per rank, train_ode with the
# YAML's dopri5 (tol 1e-3), backbone + Cayley maps + Adam, hipGraph replay
import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402
B, S = 1024, 1024
mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5", h_sample=S)
opt = mod.configure_optimizers(capturable=True)[0][0]
gx = torch.Generator(device="cpu").manual_seed(7)
x = torch.rand(B, 3, 32, 32, generator=gx).to(dev)
yb = torch.randint(0, 10, (B,), generator=gx).to(dev)
gs = GraphTrainStep(mod, opt, x, yb, warmup=2)
for _ in range(2):
    gs.step()
torch.cuda.synchronize()
a, b = ev(), ev(); a.record()
for _ in range(5):
    loss = gs.step()
b.record(); torch.cuda.synchronize()
ms = a.elapsed_time(b) / 5
st = mod.last_ode_plan["stats"].cpu().tolist()
out["train_step_B1024_S1024_dopri5"] = {"ms": round(ms, 3), "images_per_s": round(B / (ms * 1e-3), 1),
                                        "rows": B * S, "loss_finite": bool(torch.isfinite(loss)),
                                        "train_ode": {"nfe": st[0], "n_accept": st[4], "n_reject": st[5],
                                                      "status": st[3]}}
print(out["train_step_B1024_S1024_dopri5"], flush=True)
print(json.dumps(out))
