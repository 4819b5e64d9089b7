"""Standalone timing of fiode_gemm against the library GEMM (torch.matmul -> hipBLASLt) on the
configs[1] step's Cayley-layer products (tools/probes; not a test).  For each shape: mean us per
launch over `reps` back-to-back launches (HIP events), TFLOP/s, and a split-K sweep.
usage: python tools/probes/gemm_probe.py [reps]"""
import ctypes as ct
import json
import os
import sys

import torch

sys.path.insert(0, "fi-ode_amd")
from fiode_amd import ops, _lib as L  # noqa: E402

SHAPES = [  # name, M, K, N, form (see tests/test_gpu_gemm.py)
    ("G=W2 W2^T", 512, 3584, 512, "view"),
    ("P=inv^T W2", 512, 512, 3584, "At_B"),
    ("P2=inv gQ2", 512, 512, 3584, "A_B"),
    ("y1=h Q1^T", 128, 4096, 512, "A_Bt"),
    ("y2=z1 Q2^T", 128, 512, 512, "A_Bt"),
    ("dh=g1 Q1", 128, 512, 4096, "A_B"),
    ("g2 Q2", 128, 512, 512, "A_B"),
    ("dW1=g1^T h", 512, 128, 4096, "At_B"),
    ("dW2=g2^T z1", 512, 128, 512, "At_B"),
    ("dW3=g^T z2", 10, 128, 512, "At_B"),
    ("GMn 512^3", 512, 512, 512, "A_B"),
]


def operands(M, K, N, form, dev):
    if form == "view":
        W = torch.randn(M, K + 512, device=dev)
        A = W[:, 512:]
        return A, A.mT
    if form == "At_B":
        return torch.randn(K, M, device=dev).t(), torch.randn(K, N, device=dev)
    if form == "A_Bt":
        return torch.randn(M, K, device=dev), torch.randn(N, K, device=dev).t()
    return torch.randn(M, K, device=dev), torch.randn(K, N, device=dev)


def timeit(fn, reps):
    """Mean us per launch of fn() inside a captured graph of 20 launches (no host overhead)."""
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(20):
            fn()
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    n = max(1, reps // 20)
    e0.record()
    for _ in range(n):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (20 * n)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    rows = []
    for name, M, K, N, form in SHAPES:
        A, B = operands(M, K, N, form, dev)
        out = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * K
        t_lib = timeit(lambda: torch.matmul(A, B), reps)
        t_own = timeit(lambda: ops.mm(A, B, out=out), reps)
        err = float((out.double() - A.double() @ B.double()).abs().max())
        la, lb = ops._mat_layout(A), ops._mat_layout(B)
        d = L.GemmDesc(1, M, N, K, la[0], lb[0], la[1], lb[1], N, 0, 0, 0, 1.0, 0.0, 0)
        S = L.lib().fiode_gemm_splits(ct.byref(d))
        sweep = {}
        for s in (1, 2, 4, 8):
            if s > (K + 31) // 32:
                continue
            sweep[s] = round(timeit(lambda: ops.mm(A, B, out=out, split_k=s), reps), 2)
        for v in [int(t) for t in os.environ.get("GEMM_PROBE_VARIANTS", "1,2,3,5").split(",")]:
            os.environ["FIODE_GEMM_VARIANT"] = str(v)
            sweep[f"v{v}"] = round(timeit(lambda: ops.mm(A, B, out=out), reps), 2)
            os.environ["FIODE_GEMM_VARIANT"] = "0"
        r = dict(name=name, M=M, K=K, N=N, lib_us=round(t_lib, 2), own_us=round(t_own, 2), auto_split=S,
                 lib_tf=round(fl / t_lib / 1e6, 1), own_tf=round(fl / t_own / 1e6, 1), max_err=err, sweep=sweep)
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
