"""Standalone timing of fiode_cgemm vs torch.matmul (hipBLASLt) on the spectral convs' products
(not a test): median of 200 launches per shape, HIP events."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

from fiode_amd import ops  # noqa: E402

SHAPES = [("conv1 fwd", 544, 32, 128, 3, False), ("conv2 fwd", 144, 32, 128, 128, False),
          ("conv3 fwd", 144, 64, 128, 32, False), ("conv4 fwd", 40, 64, 128, 256, False),
          ("conv4 dX", 40, 256, 128, 64, True), ("conv3 dX", 144, 32, 128, 64, True),
          ("conv2 dX", 144, 128, 128, 32, True)]


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


dev = torch.device("cuda:0")
for name, F, M, N, K, ca in SHAPES:
    A = torch.randn((F, K, M) if ca else (F, M, K), dtype=torch.complex64, device=dev)
    B = torch.randn((F, K, N), dtype=torch.complex64, device=dev)
    t_own = timeit(lambda: ops.cgemm(A, B, conj_trans_a=ca))
    t_lib = timeit(lambda: torch.matmul(A.mH if ca else A, B))
    fl = 8.0 * F * M * N * K
    print(f"{name:10s} F={F:4d} M={M:4d} N={N} K={K:4d}: cgemm {t_own:6.1f} us ({fl / t_own / 1e6:6.1f} TF/s), "
          f"library {t_lib:6.1f} us", flush=True)
