"""Probe (not a test): the one-launch block inverse (cayley.hip k_pinv) stage by stage for n = 64 NB:
the published pivot inverses P_k and tile versions in the workspace against float64 recomputations,
and the output per 64 x 64 tile.  python tools/probes/pinv_probe.py [n ...]"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

from fiode_amd import ops, _lib as L  # noqa: E402

dev = torch.device("cuda:0")


def acc_layout(t):           # [64, 64] -> the kernel's f4 order (e = (4 w + bj) 64 + lane, rows 16w+4q+r, col 16bj+i)
    out = torch.empty(1024, 4, dtype=t.dtype)
    for e in range(1024):
        w, bj, ln = e >> 8, (e >> 6) & 3, e & 63
        q, i = ln >> 4, ln & 15
        out[e] = t[16 * w + 4 * q: 16 * w + 4 * q + 4, 16 * bj + i]
    return out.reshape(-1)


for n in [int(a) for a in sys.argv[1:]] or [128, 256, 512]:
    NB = n // 64
    g = torch.Generator().manual_seed(n)
    A = torch.randn(n, n, generator=g, dtype=torch.float64) * (1.0 / n ** 0.5)
    M = torch.eye(n, dtype=torch.float64) + (A - A.T) + 0.3 * A.T @ A
    Md = M.float().to(dev)
    out = torch.empty_like(Md)
    nbytes = L.lib().fiode_block_inverse_workspace_bytes(n)
    ws = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
    for rep in range(3):      # the same workspace again: the kernel must leave it ready
        out.fill_(0.0)
        rc = L.lib().fiode_block_inverse(ops._stream(dev), n, Md.data_ptr(), out.data_ptr(), ws.data_ptr(), nbytes)
        torch.cuda.synchronize()
        print(f"  call {rep}: max err {float((out.double().cpu() - torch.linalg.inv(M)).abs().max()):.3e}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.lib().fiode_block_inverse(ops._stream(dev), n, Md.data_ptr(), out.data_ptr(), ws.data_ptr(), nbytes)
    e1.record()
    torch.cuda.synchronize()
    print(f"  {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call (20 back to back)")
    ref = torch.linalg.inv(M)
    err = (out.double().cpu() - ref).abs()
    print(f"n={n} rc={rc} max err {float(err.max()):.3e}", flush=True)
    for ti in range(NB):
        print("  tile row", ti, [f"{float(err[64*ti:64*ti+64, 64*tj:64*tj+64].max()):.1e}" for tj in range(NB)])
    nflag = NB ** 3 + NB + 1
    fl = ws[:nflag].view(torch.int32).cpu()
    print("  flags after the call (must be 0):", int((fl != 0).sum()))
    # pivot inverses: recompute in float64 by plain block elimination
    X = M.clone()
    Ps = []
    for k in range(NB):
        K = slice(64 * k, 64 * k + 64)
        P = torch.linalg.inv(X[K, K])
        Ps.append(P)
        R = P @ X[K, :]
        C = X[:, K].clone()
        X -= C @ R
        X[K, :] = R
        X[:, K] = -(C @ P)
        X[K, K] = P
    flag_floats = (nflag + 63) // 64 * 64
    Pt = ws[flag_floats + NB * NB * NB * 4096: flag_floats + NB * NB * NB * 4096 + NB * 4096].cpu().double()
    for k in range(NB):
        got = Pt[4096 * k: 4096 * (k + 1)]
        print(f"  P_{k}: max |published - float64| {float((got - acc_layout(Ps[k])).abs().max()):.3e}, "
              f"max |P| {float(Ps[k].abs().max()):.3e}, published zeros {int((got == 0).sum())}")

# n = 128: which formula does the wrong tile (0, 1) follow?
n = 128
g = torch.Generator().manual_seed(n)
A = torch.randn(n, n, generator=g, dtype=torch.float64) * (1.0 / n ** 0.5)
M = torch.eye(n, dtype=torch.float64) + (A - A.T) + 0.3 * A.T @ A
Md = M.float().to(dev)
out = torch.empty_like(Md)
nbytes = L.lib().fiode_block_inverse_workspace_bytes(n)
ws = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
L.lib().fiode_block_inverse(ops._stream(dev), n, Md.data_ptr(), out.data_ptr(), ws.data_ptr(), nbytes)
torch.cuda.synchronize()
o = out.double().cpu()[0:64, 64:128]
K0, K1 = slice(0, 64), slice(64, 128)
P0 = torch.linalg.inv(M[K0, K0])
S = M[K1, K1] - M[K1, K0] @ P0 @ M[K0, K1]
P1 = torch.linalg.inv(S)
cands = {"correct": -(P0 @ M[K0, K1]) @ P1, "-in01 P1": -M[K0, K1] @ P1, "-(P0 in01) P0": -(P0 @ M[K0, K1]) @ P0,
         "P0 in01": P0 @ M[K0, K1], "zeros": torch.zeros(64, 64, dtype=torch.float64), "in01": M[K0, K1],
         "-(P0 in01)": -(P0 @ M[K0, K1]), "(P0 in01) P1": (P0 @ M[K0, K1]) @ P1}
for k, v in cands.items():
    print(f"tile(0,1) vs {k}: {float((o - v).abs().max()):.3e}")
print("tile(0,1) sample", o[0, :4].tolist(), "correct", cands["correct"][0, :4].tolist())
err = (o - cands["correct"]).abs()
print("tile(0,1) error by 16x16 block (rows = 16 w .., cols = 16 bj ..):")
for w in range(4):
    print("   ", [f"{float(err[16*w:16*w+16, 16*b:16*b+16].max()):.1e}" for b in range(4)])
bad = (err > 1e-4).nonzero()
print("bad elements", bad.shape[0], "first", bad[:8].tolist())
rows = sorted({int(r) for r, c in bad.tolist()})
print("bad rows", rows)
m = err > 1e-4
for k in ([] if not bool(m.any()) else ("correct", "(P0 in01) P1", "P0 in01", "-(P0 in01)")):
    print(f"  at the bad elements vs {k}: {float((o[m] - cands[k][m]).abs().max()):.3e}")
print("  values", o[3, 48:52].tolist(), "correct", cands["correct"][3, 48:52].tolist())

# phase timestamps of the n = 512 chain (fiode_debug_pinv_profile)
import ctypes as ct  # noqa: E402
n = 512
g = torch.Generator().manual_seed(n)
A = torch.randn(n, n, generator=g, dtype=torch.float64) * (1.0 / n ** 0.5)
M = (torch.eye(n, dtype=torch.float64) + (A - A.T) + 0.3 * A.T @ A).float().to(dev)
out = torch.empty_like(M)
nbytes = L.lib().fiode_block_inverse_workspace_bytes(n)
ws = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
prof = torch.zeros(2048, dtype=torch.int64, device=dev)
fn = L.lib().fiode_debug_pinv_profile
fn.argtypes = [ct.c_void_p, ct.c_int32, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
for _ in range(3):
    L.lib().fiode_block_inverse(ops._stream(dev), n, M.data_ptr(), out.data_ptr(), ws.data_ptr(), nbytes)
torch.cuda.synchronize()
assert fn(ops._stream(dev), n, M.data_ptr(), out.data_ptr(), ws.data_ptr(), prof.data_ptr()) == 0
torch.cuda.synchronize()
p = prof.cpu().tolist()
t0 = min(p[1024:1024 + 65])
us = lambda v: (v - t0) / 100.0
print("WG start spread (us): first", us(min(p[1024:1089])), "last", us(max(p[1024:1089])))
for k in range(8):
    print(f"chain k={k}: invert {us(p[8*k]):7.2f} -> {us(p[8*k+1]):7.2f}  published {us(p[8*k+2]):7.2f}  "
          f"next D ready {us(p[8*k+3]) if k < 7 else float('nan'):7.2f}")
ends = [[us(p[256 + t * 8 + k]) for k in range(8)] for t in range(64)]
for k in range(8):
    col = [ends[t][k] for t in range(64) if p[256 + t * 8 + k]]
    print(f"tiles step {k}: first end {min(col):7.2f} last end {max(col):7.2f}")
