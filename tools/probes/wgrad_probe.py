"""Per-workgroup phase stamps of k_lyap_wgrad in the train_ode backward (needs tools/libfiode_prof.so,
`make -C fi-ode_amd/csrc prof`; not a test): start -> rows staged in LDS -> MFMA done -> slab stored,
wall clock (100 MHz), over the bench's captured configs[1] step."""
import ctypes as ct
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
os.environ["FIODE_LIB"] = str(ROOT / "tools" / "libfiode_prof.so")
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import _lib as L  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
mod = bench.build_module(dev, seed=0, train_ode=True, solver="rk4")
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
gs = GraphTrainStep(mod, opt, x, y)
for _ in range(6):
    gs.step()
torch.cuda.synchronize()
buf = (ct.c_ulonglong * 4096)()
lib = L.lib()
lib.fiode_debug_wgrad_stamps.argtypes = [ct.c_void_p, ct.c_int]
assert lib.fiode_debug_wgrad_stamps(buf, 4096) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4).astype(np.float64) * 0.01
st = st[st[:, 3] > 0]
t0 = st[:, 0].min()
print(f"k_lyap_wgrad: {len(st)} workgroups, span {st[:, 3].max() - t0:.2f} us; start offsets p50/max "
      f"{np.median(st[:, 0] - t0):.2f} / {(st[:, 0] - t0).max():.2f}")
for k, name in ((1, "stage"), (2, "mfma"), (3, "slab store")):
    d = st[:, k] - st[:, k - 1]
    print(f"  {name}: p10/p50/p90/max {np.percentile(d, 10):.2f} / {np.median(d):.2f} / {np.percentile(d, 90):.2f} / {d.max():.2f} us")
gs.close()
