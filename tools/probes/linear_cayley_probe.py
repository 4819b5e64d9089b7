"""Kernel composition of the dense Cayley maps (backbone CayleyLinears + dynamics) fwd + bwd
(not a test): run under rocprofv3 --kernel-trace --stats; 20 iterations."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.cayley import CayleyLinear  # noqa: E402

dev = torch.device("cuda:0")
mod = bench.build_module(dev, train_ode=True)
which = sys.argv[1] if len(sys.argv) > 1 else "all"
lins = [m for m in mod.init_coordinates.modules() if isinstance(m, CayleyLinear)]
dyn = mod.dyn_fun
for _ in range(20):
    if which in ("all", "lin"):
        for m in lins:
            Q = m.effective_weight()
            Q.backward(torch.ones_like(Q))
    if which in ("all", "dyn"):
        w = dyn._effective_weights()
        sum(v.sum() for v in w.values()).backward()
torch.cuda.synchronize()
print("ok")
