"""Is the replayed step bound by the GPU or by hipGraph submission? (not a test)
Times the host side of CUDAGraph.replay() against the GPU completion of the same replays."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
for ode in (True, False):
    mod = bench.build_module(dev, train_ode=ode)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    x = torch.rand(128, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    gs = GraphTrainStep(mod, opt, x, y)
    for _ in range(5):
        gs.step()
    torch.cuda.synchronize()
    n = 30
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        gs.g_fb.replay()
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print(f"ode={ode}: host replay() median {host[n // 2] * 1e3:.3f} ms, enqueue loop {(t1 - t0) / n * 1e3:.3f} ms/step, "
          f"wall {(t2 - t0) / n * 1e3:.3f} ms/step", flush=True)
    # GPU time of one replay with the host far ahead
    torch.cuda._sleep(100_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        gs.g_fb.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"ode={ode}: GPU ms per replay behind a sleep {e0.elapsed_time(e1) / 10:.3f}", flush=True)
