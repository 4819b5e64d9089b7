"""Probe (not a test): capture the configs[1] training step (GraphTrainStep, bench.py's module) and
replay it under the queue settings the environment gives (GPU_MAX_HW_QUEUES,
DEBUG_HIP_FORCE_GRAPH_QUEUES; read by the HIP runtime at initialisation), with a native backtrace on
SIGSEGV (tools/native/libsegv_bt.so) and Python's faulthandler (all threads), so a host fault
inside the runtime names its frames.  Every phase prints a line before it starts, so a fault names
its phase too:
  1. streams: a normal and a priority -1 stream (the ODE solve's), a tiny two-branch graph captured
     on them and replayed -- the runtime primitives alone;
  2. warm-up + capture of the bench step (GraphTrainStep with bench.py's placement trials);
  3. replays.

python tools/probes/graph_queue_probe.py [replays] [placement_trials]
"""
import ctypes
import faulthandler
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
faulthandler.enable(all_threads=True)
ctypes.CDLL(str(ROOT / "tools" / "native" / "libsegv_bt.so"))

import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda:0")
print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"), "DEBUG_HIP_FORCE_GRAPH_QUEUES =",
      os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES"), flush=True)

print("phase 1: streams + two-branch graph", flush=True)
a = torch.ones(1 << 20, device=dev)
s_lo, s_hi = torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=-1)
g1 = torch.cuda.CUDAGraph()
cap = torch.cuda.Stream(dev)
with torch.cuda.graph(g1, stream=cap, capture_error_mode="thread_local"):
    cur = torch.cuda.current_stream()
    for s in (s_lo, s_hi):
        s.wait_stream(cur)
    with torch.cuda.stream(s_lo):
        b = a * 2.0
    with torch.cuda.stream(s_hi):
        c = a + 1.0
    cur.wait_stream(s_lo)
    cur.wait_stream(s_hi)
    d = b + c
for _ in range(10):
    g1.replay()
torch.cuda.synchronize()
print("phase 1 ok:", float(d[0]), flush=True)

print(f"phase 2: warm-up + capture (placement trials {trials})", flush=True)
mod = bench.build_module(dev, seed=0, train_ode=True)
opt = mod.configure_optimizers(capturable=True)[0][0]
g = torch.Generator(device="cpu").manual_seed(1234)
x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
y = torch.randint(0, 10, (128,), generator=g).to(dev)
t0 = time.time()
gs = GraphTrainStep(mod, opt, x, y, placement_trials=trials)
print(f"captured in {time.time() - t0:.1f} s, placement {gs.placement_ms}", flush=True)
print("phase 3: replays", flush=True)
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
