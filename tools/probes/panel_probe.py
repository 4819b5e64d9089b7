"""k_panel_update latency alone / two chains / beside a busy stream, as hipGraph replays (not a test).
Run under rocprofv3 --kernel-trace for per-kernel durations; prints us per replay per case."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402
from fiode_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def graph_us(fn, reps=30):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 2)


A = torch.randn(512, 512, device=dev) * 0.05
M1 = torch.eye(512, device=dev) + (A - A.T)
M2 = M1.clone()
X = torch.randn(4096, 4096, device=dev)
side = [torch.cuda.Stream() for _ in range(2)]


def two():
    cur = torch.cuda.current_stream()
    for s in side:
        s.wait_stream(cur)
    with torch.cuda.stream(side[0]):
        ops.block_inverse(M1)
    with torch.cuda.stream(side[1]):
        ops.block_inverse(M2)
    for s in side:
        cur.wait_stream(s)


def with_gemm():
    cur = torch.cuda.current_stream()
    side[0].wait_stream(cur)
    with torch.cuda.stream(side[0]):
        ops.block_inverse(M1)
    for _ in range(4):
        torch.matmul(X, X)
    cur.wait_stream(side[0])


res = {"one": graph_us(lambda: ops.block_inverse(M1)), "two": graph_us(two),
       "gemm4_alone": graph_us(lambda: [torch.matmul(X, X) for _ in range(4)]), "inv_with_gemm4": graph_us(with_gemm)}
print(json.dumps(res), flush=True)
