"""Latency of the dense Cayley maps' small fp32 GEMMs as hipGraph replays, library tile choice vs
column-split batched forms (not a test).  python tools/probes/gemm_probe.py -> one JSON line."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def graph_us(fn, reps=50):
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


A = torch.randn(512, 512, device=dev)
B = torch.randn(512, 512, device=dev)
W = torch.randn(512, 3584, device=dev)
res = {}
res["mm512"] = graph_us(lambda: torch.matmul(A, B))
res["mm512_T"] = graph_us(lambda: torch.matmul(A.mT, B))
for nb in (2, 4, 8):
    Bs = B.reshape(512, nb, 512 // nb).permute(1, 0, 2).contiguous()      # [nb, 512, 512/nb]
    res[f"bmm512_split{nb}"] = graph_us(lambda: torch.matmul(A, Bs))
    As = A.reshape(nb, 512 // nb, 512).contiguous()                       # row blocks
    res[f"bmm512_rows{nb}"] = graph_us(lambda: torch.matmul(As, B))
res["chain2_512"] = graph_us(lambda: torch.matmul(A.mT, torch.matmul(B, A.mT)))
res["wide_512x3584"] = graph_us(lambda: torch.matmul(A.mT, W))
for nb in (4, 8):
    As = A.mT.reshape(nb, 512 // nb, 512)
    res[f"wide_rows{nb}"] = graph_us(lambda: torch.matmul(As, W))
print(json.dumps(res), flush=True)
