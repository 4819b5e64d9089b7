"""Standalone timing of the linear head's library GEMMs in alternative forms (not a test): the
first layer's input gradient dh = g1 Q1 ([128 x 512] x [512 x 4096]) and forward h Q1^T + b, median
of 200 launches, HIP events.  (r05cj also timed a 32 x 32-tile f32 MFMA kernel for dh: 18.7 vs 28.6 us
with the events, step unchanged in the A/B -- removed; profiles/r05cj.)"""
import torch

dev = torch.device("cuda:0")


def timeit(fn, reps=200):
    for _ in range(20):
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


g1 = torch.randn(128, 512, device=dev)
Q1 = torch.randn(512, 4096, device=dev)
h = torch.randn(128, 4096, device=dev)
b1 = torch.randn(512, device=dev)
Q1t = Q1.t().contiguous()
empty = timeit(lambda: None)
forms = {
    "dh = g1.mm(Q1)": lambda: g1.mm(Q1),
    "dh = (Q1^T g1^T)^T contiguous": lambda: torch.mm(Q1.t(), g1.t()).t().contiguous(),
    "dh = (Q1^T g1^T)^T (view)": lambda: torch.mm(Q1.t(), g1.t()),
    "dh = g1.mm(Q1t^T) (Q1 stored transposed)": lambda: g1.mm(Q1t.t()),
    "fwd addmm(b1, h, Q1^T)": lambda: torch.addmm(b1, h, Q1.t()),
    "fwd h.mm(Q1t) + b1 (Q1 stored transposed)": lambda: torch.addmm(b1, h, Q1t),
    "fwd (Q1 h^T)^T": lambda: torch.mm(Q1, h.t()),
    "dW1 = g1^T h": lambda: g1.t().mm(h),
}
print(f"empty event pair: {empty:.1f} us")
for k, f in forms.items():
    print(f"{k:45s} {timeit(f):7.1f} us", flush=True)
