"""configs[4]'s captured training step (B = 1,024 x S = 1,024, train_ode dopri5 tol 1e-3) replayed a
few times, for a rocprofv3 --kernel-trace --stats breakdown of where its ~7.4 ms go.  Prints the
replay time from HIP events.  (tools; not a test)

usage: rocprofv3 --kernel-trace --stats -d <dir> -o run -- python tools/probes/large_step_trace.py [replays] [modes]
modes (comma list, default "side"): side = the solve on its own stream beside the fan-out (the
product), serial = the solve on the step's stream (ode_side_stream False); alternated 3 rounds.
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
modes = (sys.argv[2] if len(sys.argv) > 2 else "side").split(",")
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(1024, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (1024,), generator=g).to(dev)
steps = {}
for mode in modes:
    mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5", h_sample=1024)
    mod.ode_side_stream = mode != "serial"
    opt = mod.configure_optimizers(capturable=True)[0][0]
    steps[mode] = GraphTrainStep(mod, opt, x, y, placement_trials=1)
times = {m: [] for m in modes}
for r in range(3):
    for mode, gs in steps.items():
        for _ in range(3):
            gs.step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            gs.step()
        e1.record()
        torch.cuda.synchronize()
        times[mode].append(round(e0.elapsed_time(e1) / n, 4))
print(json.dumps({"replays": n, "ms_per_step": times,
                  "skipped": {m: gs.skipped_steps() for m, gs in steps.items()}}), flush=True)
for gs in steps.values():
    gs.close()
