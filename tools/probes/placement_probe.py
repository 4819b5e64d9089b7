"""Is the captured step's time a function of the streams it was captured on? (not a test)

python tools/probes/placement_probe.py  ->  one JSON line of ms per step

The same module and batch captured several ways, each timed over the same replay count:
  first       GraphTrainStep as bench.py builds it
  recapture   gs._capture() again: every stream object the same
  new_gs      a second GraphTrainStep on the module (side / ODE streams kept; conv map streams new)
  fresh_k     the module's side and ODE streams dropped first (new pool streams), k = 0..3
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
mod = bench.build_module(dev, train_ode=True)
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)


def timed(gs, reps=3, n=30):
    out = []
    for _ in range(reps):
        for _ in range(3):
            gs.step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            gs.step()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t) / n * 1e3)
    return round(min(out), 4)


res = {}
gs = GraphTrainStep(mod, opt, x, y)
res["first"] = timed(gs)
gs._capture()
res["recapture"] = timed(gs)
gs._capture()
res["recapture2"] = timed(gs)
gs.close()
gs = GraphTrainStep(mod, opt, x, y)
res["new_gs"] = timed(gs)
for k in range(4):
    gs.close()
    mod._side_streams = None
    mod._ode_stream = None
    gs = GraphTrainStep(mod, opt, x, y)
    res[f"fresh_{k}"] = timed(gs)
    gs._capture()
    res[f"fresh_{k}_recap"] = timed(gs)
print(json.dumps(res), flush=True)
