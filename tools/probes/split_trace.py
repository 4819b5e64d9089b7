"""Replays of the configs[1] step for a rocprofv3 kernel trace (not a test):
python tools/probes/split_trace.py split|one|serial  (15 replays after the capture)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import graph_step as GS  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "split"
if mode == "serial":
    GS.D_CHAINS = False
dev = torch.device("cuda:0")
mod = bench.build_module(dev, seed=0, train_ode=True)
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
gs = GS.GraphTrainStep(mod, opt, x, y, split=(mode != "one"))
for _ in range(15):
    gs.step()
torch.cuda.synchronize()
print(mode, "split", gs.split, flush=True)
