"""configs[4] (B = 1,024 x S = 1,024, train_ode dopri5 tol 1e-3): how many replays the step guard skips
on a NaN loss when every replay trains on the same synthetic batch (bench.py's companion) vs a
rotating pool of distinct synthetic batches copied into the graph's static inputs (what a data
loader does).  Prints one JSON line per mode.  (tools; not a test)

usage: python tools/probes/large_batch_probe.py [replays] [pool]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "fi-ode_amd"))
import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
pool = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for mode in ("same", "rotate"):
    mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5", h_sample=1024)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    xs = [torch.rand(1024, 3, 32, 32, generator=g).to(dev) for _ in range(pool)]
    ys = [torch.randint(0, 10, (1024,), generator=g).to(dev) for _ in range(pool)]
    gs = GraphTrainStep(mod, opt, xs[0], ys[0], placement_trials=1)
    finite = []
    for i in range(n):
        if mode == "rotate":
            loss = gs.step(xs[i % pool], ys[i % pool])
        else:
            loss = gs.step()
        torch.cuda.synchronize()
        finite.append(bool(torch.isfinite(loss).all()))
    print(json.dumps({"mode": mode, "replays": n, "pool": pool if mode == "rotate" else 1,
                      "finite": finite, "skipped": gs.skipped_steps()}), flush=True)
    gs.close()
    del gs, mod, opt
    torch.cuda.empty_cache()
