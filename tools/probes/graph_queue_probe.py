"""Probe (not a test): capture the configs[1] training step (GraphTrainStep, bench.py's module) and
replay it under the graph-executor setting the environment gives (DEBUG_HIP_FORCE_GRAPH_QUEUES, read
by the HIP runtime at initialisation), with a native backtrace on SIGSEGV (tools/native/libsegv_bt.so)
and Python's faulthandler, so a host fault inside the runtime names its frames.

python tools/probes/graph_queue_probe.py [replays]
"""
import ctypes
import faulthandler
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
faulthandler.enable()
ctypes.CDLL(str(ROOT / "tools" / "native" / "libsegv_bt.so"))

import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda:0")
print("DEBUG_HIP_FORCE_GRAPH_QUEUES =", os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES"), flush=True)
mod = bench.build_module(dev, seed=0, train_ode=True)
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
t0 = time.time()
gs = GraphTrainStep(mod, opt, x, y)
print(f"captured in {time.time() - t0:.1f} s", flush=True)
losses = []
for i in range(reps):
    losses.append(gs.step().detach().clone())
    if i < 3:
        torch.cuda.synchronize()
        print("replay", i, "ok", flush=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    gs.step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20 * 1e3
L = torch.stack(losses)
print(f"ok: {reps} replays, losses finite {bool(torch.isfinite(L).all())}, status {mod.device_status()}, "
      f"{dt:.3f} ms/step", flush=True)
