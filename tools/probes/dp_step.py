"""The configs[2] step (train_ode with dopri5, B=128, S=256) as a captured hipGraph, replayed N times
(not a test) -- for rocprofv3 kernel traces of the dopri5 training step.
python tools/probes/dp_step.py [replays]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5")
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
gs = GraphTrainStep(mod, opt, x, y)
for _ in range(3):
    gs.step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    gs.step()
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t) / reps * 1e3:.3f} ms per step; last solve stats "
      f"{mod.last_ode_plan['stats'].cpu().tolist()}", flush=True)
gs.close()
