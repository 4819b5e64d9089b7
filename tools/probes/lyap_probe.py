"""Phase timing of the fan-out kernels k_lyap_fwd / k_lyap_bwd (needs tools/libfiode_prof.so, built
with -DOT_PROFILE by `make -C fi-ode_amd/csrc prof`; not a test).  Every wave's lane 0 adds its
wall-clock ticks (100 MHz) per phase; printed as the mean per wave in microseconds."""
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
os.environ["FIODE_LIB"] = str(ROOT / "tools" / "libfiode_prof.so")
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import ctypes as ct  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fiode_amd import _lib as L, ops  # noqa: E402
from tests._util import make_params  # noqa: E402

dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
B, S = 128, 256
g = torch.Generator().manual_seed(0)
x = torch.randn(B, 10, generator=g).to(dev)
y = torch.randint(0, 10, (B,), generator=g).to(dev)
dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(L.LYAP_KERNELS) + 1)]
for rep in range(4):
    ops.lyap_step(x, y, w, dyn, sample_size=S, n_uniform=204, seed=1, offset=rep, events=ev)
torch.cuda.synchronize()
print("kernel us (last rep, alone on the GPU):",
      {k: round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i, k in enumerate(L.LYAP_KERNELS)})
lib = L.lib()
cfg = L.LyapConfig(B, S, 204, L.FIODE_SAMPLER_COMPOSITE, L.FIODE_DROPOUT_PHILOX, 2.0, 1, 3)
nb = lib.fiode_lyap_workspace_bytes(ct.byref(cfg), ct.byref(dyn.to_c()))
ws = ops._Workspace.get(dev, nb, "lyap")
allp = ws[nb - (64 + 4096) * 8:nb].view(torch.int64).cpu().numpy()
prof = allp[:64]
for name, base, nwg in (("k_lyap_fwd", 64, 512), ("k_lyap_bwd", 64 + 2048, 256)):
    st = allp[base:base + 2 * nwg].reshape(nwg, 2).astype(np.float64) * 0.01
    st = st[st[:, 1] > 0]                      # the launched workgroups (the grid may be smaller)
    nwg = len(st)
    t0 = st[:, 0].min()
    dur = st[:, 1] - st[:, 0]
    print(f"{name}: span {st[:, 1].max() - t0:.1f} us; workgroup start offsets (us) p50 {np.median(st[:, 0] - t0):.1f} "
          f"max {(st[:, 0] - t0).max():.1f}; durations p10/p50/p90/max {np.percentile(dur, 10):.1f} / "
          f"{np.median(dur):.1f} / {np.percentile(dur, 90):.1f} / {dur.max():.1f}")
    slow = np.argsort(dur)[::-1][:6]
    print(f"  slowest workgroups (id: start offset, duration us): "
          + ", ".join(f"{i}: {st[i, 0] - t0:.1f}, {dur[i]:.1f}" for i in slow))
fw, bw = max(int(prof[6]), 1), max(int(prof[18]), 1)
us = lambda i, n: prof[i] / n * 0.01
print(f"k_lyap_fwd ({fw} waves), us per wave: weights {us(0, fw):.2f}  row loads {us(1, fw):.2f}  "
      f"MLP {us(2, fw):.2f}  ft+nominal {us(3, fw):.2f}  QP {us(4, fw):.2f}  stores {us(5, fw):.2f}")
print(f"k_lyap_bwd ({bw} waves), us per wave: weights {us(8, bw):.2f}  phase A (QP rows) {us(9, bw):.2f}  "
      f"L1+L2+ga {us(10, bw):.2f}  barrier {us(11, bw):.2f}  gb {us(12, bw):.2f}  barrier {us(13, bw):.2f}  "
      f"wgrad {us(14, bw):.2f}  g_u {us(15, bw):.2f}  barrier {us(16, bw):.2f}  partial adds {us(17, bw):.2f}")
