"""Kernel timings of the throughput kernels for one library build (not a test): the fused fan-out
(fiode_lyap_step at B=128, S=256, per-kernel HIP events, median of 20) and the certification of
one image on the T=40 grid (fiode_certify, median of 3).  FIODE_LIB selects the build.
usage: python tools/ab_fanout.py [tag] [--large] [--no-cert]  -> one JSON line
(--large adds the fan-out at B=1024, S=1024: BASELINE configs[4]'s fan-out on one GPU)"""
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
tag = args[0] if args else "lib"
dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
B, S = 128, 256
g = torch.Generator().manual_seed(0)
x = torch.randn(B, 10, generator=g).to(dev)
y = torch.randint(0, 10, (B,), generator=g).to(dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
nk = len(L.LYAP_KERNELS)
per = {k: [] for k in L.LYAP_KERNELS}
for rep in range(23):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(nk + 1)]
    torch.cuda._sleep(2_000_000)
    sc, gr, _ = ops.lyap_step(x, y, w, dyn, sample_size=S, n_uniform=204, seed=1, offset=rep, events=ev)
    torch.cuda.synchronize()
    if rep >= 3:
        for i, k in enumerate(L.LYAP_KERNELS):
            per[k].append(ev[i].elapsed_time(ev[i + 1]) * 1e3)
out = {"tag": tag, "fanout_us": {k: round(statistics.median(v), 2) for k, v in per.items()},
       "loss": float(sc[0])}
if "--large" in sys.argv:
    BL, SL = 1024, 1024
    xl = torch.randn(BL, 10, generator=g).to(dev)
    yl = torch.randint(0, 10, (BL,), generator=g).to(dev)
    perl = {k: [] for k in L.LYAP_KERNELS}
    for rep in range(8):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nk + 1)]
        scl, _, _ = ops.lyap_step(xl, yl, w, dyn, sample_size=SL, n_uniform=816, seed=1, offset=rep, events=ev)
        torch.cuda.synchronize()
        if rep >= 2:
            for i, k in enumerate(L.LYAP_KERNELS):
                perl[k].append(ev[i].elapsed_time(ev[i + 1]) * 1e3)
    out["fanout_large_us"] = {k: round(statistics.median(v), 2) for k, v in perl.items()}
    out["loss_large"] = float(scl[0])
if "--no-cert" in sys.argv:
    print(json.dumps(out), flush=True)
    sys.exit(0)
grid = ops.certify_grid(40, device=dev)
xf = torch.randn(10, generator=g).to(dev)
cd = ops.DynCfg(scale_nominal=False, dropout=0.0)
ops.certify_image(xf, 3, grid, w, cd, T=40, batches=10)
torch.cuda.synchronize()
ts = []
for lab in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    o, it = ops.certify_image(xf, lab, grid, w, cd, T=40, batches=10)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = statistics.median(ts)
G = int(grid.shape[0])
out["certify_ms_per_image"] = round(ms, 3)
out["certify_mlp_tflops"] = round(37888 * G / (ms * 1e-3) / 1e12, 2)
out["certify_max_viol"] = [round(float(v), 5) for v in o[:, 0].cpu()]
print(json.dumps(out), flush=True)
