"""Cayley-orthogonal layers (host side, PyTorch-ROCm).

The reference imports ``CayleyLinear``, ``CayleyConv`` and ``GroupSort`` from the
``libs/ortho_conv`` submodule, which is empty in the reference tree.
The only in-tree statement of the parametrisation is ``convert_cayley``
(dynamics/classification.py:281-294): Q = cayley(alpha * W / ||W||) with the bias kept apart.
This module restates the public orthogonal-convolutions design (Trockman & Kolter, ICLR 2021):
parity with the absent submodule is unpinned; orthogonality is tested (Q^T Q = I).

These maps are tiny per-step parameter transforms (10x10 and 128x128 inverses for the dynamics)
and stay in PyTorch: their gradients come from autograd, fed by the fused HIP step's dL/dQ.
"""
from __future__ import annotations

import ctypes as ct
import math
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .streams import new_stream


_BLOCK = 128


def _block_inverse(M: torch.Tensor) -> torch.Tensor:
    """Inverse of (..., n, n) on the device: real n > 64 by the 64-panel block Gauss-Jordan kernels
    (fiode_block_inverse), n <= 128 otherwise by the register Gauss-Jordan kernel, complex n > 128
    by block Gauss-Jordan in natural order over 128-wide panels here (pivot blocks inverted by the
    kernel, the rank-128 updates as batched GEMMs).  Valid for positive-real matrices (every
    Schur complement of one is positive-real), which all Cayley systems I + A are."""
    from . import ops
    n = M.shape[-1]
    if n > 64 and M.dtype == torch.float32 and M.is_cuda:
        if M.dim() == 2:
            return ops.block_inverse(M)
        return ops.block_inverse(M.reshape(-1, n, n)).reshape(M.shape)
    if n <= _BLOCK:
        return ops.batched_inverse(M)
    X = M.clone()
    for k0 in range(0, n, _BLOCK):
        K = slice(k0, min(n, k0 + _BLOCK))
        P = ops.batched_inverse(X[..., K, K])
        R = P @ X[..., K, :]                     # pivot block row, scaled
        Cm = X[..., :, K].clone()                # pivot block column (old)
        X -= Cm @ R
        X[..., K, :] = R
        X[..., :, K] = -(Cm @ P)
        X[..., K, K] = P
    return X


class _CayleyInverse(torch.autograd.Function):
    """(I + A)^-1 with torch.linalg.inv's gradient, d(M^-1) = -M^-H dM M^-H -- computed by the
    fiode_batched_inverse kernel instead of getrf/getrs (no pivot search, no info sync)."""

    @staticmethod
    def forward(ctx, M):
        inv = _block_inverse(M.contiguous())
        ctx.save_for_backward(inv)
        return inv

    @staticmethod
    def backward(ctx, g):
        inv, = ctx.saved_tensors
        ih = inv.mH
        return -(ih @ g @ ih)


class _CayleyScaledFn(torch.autograd.Function):
    """Q = cayley(alpha * W / ||W||) with an analytic backward (one autograd node instead of the
    ~40 of the op-by-op graph).  W: [..., cout, cin] real or complex; the norm is over the whole
    tensor (``per_matrix`` False: CayleyConv's one alpha for all frequencies) or over each matrix
    (True: several same-shape linears batched, alpha [batch]).  Wide maps go through the transpose.

    Forward, with X = s W (s = alpha / ||W||), U = X[:cin], V = X[cin:]:
        M = I + U - U^H + V^H V,  inv = M^-1,  Q = [2 inv - I ; -2 V inv].
    Backward, G = dL/dQ = [Gt ; Gb]:
        G_inv = 2 Gt - 2 V^H Gb,  G_M = -inv^H G_inv inv^H,
        dL/dU = G_M - G_M^H,      dL/dV = V (G_M + G_M^H) - 2 Gb inv^H,
        D = Re<dL/dX, W>,  dL/dW = s dL/dX - alpha D / ||W||^3 W,  dL/dalpha = D / ||W||."""

    @staticmethod
    def forward(ctx, W, alpha, per_matrix: bool):
        Wd = W.detach()
        if per_matrix:
            n = torch.linalg.vector_norm(Wd, dim=(-2, -1), keepdim=True)
            s = alpha.detach().reshape(n.shape) / n
        else:
            n = torch.linalg.vector_norm(Wd)
            s = alpha.detach().reshape(()) / n
        X = Wd * s
        wide = X.shape[-1] > X.shape[-2]
        if wide:
            X = X.mT
        cin = X.shape[-1]
        tall = X.shape[-2] > cin
        U, V = X[..., :cin, :], X[..., cin:, :]
        M = U - U.mH
        if tall:
            M = M + V.mH @ V
        M.diagonal(dim1=-2, dim2=-1).add_(1.0)
        inv = _block_inverse(M.contiguous())
        top = inv * 2.0
        top.diagonal(dim1=-2, dim2=-1).sub_(1.0)
        Q = torch.cat([top, (V @ inv).mul_(-2.0)], dim=-2) if tall else top
        ctx.save_for_backward(Wd, alpha, n, s, inv, V if tall else None)
        ctx.flags = (wide, tall, per_matrix, cin)
        return Q.mT if wide else Q

    @staticmethod
    def backward(ctx, G):
        Wd, alpha, n, s, inv, V = ctx.saved_tensors
        wide, tall, per_matrix, cin = ctx.flags
        if wide:
            G = G.mT
        ih = inv.mH
        Gt = G[..., :cin, :]
        if tall:
            Gb = G[..., cin:, :]
            Ginv = 2.0 * Gt - 2.0 * (V.mH @ Gb)
        else:
            Ginv = 2.0 * Gt
        GM = -(ih @ Ginv @ ih)
        gU = GM - GM.mH
        if tall:
            gV = V @ (GM + GM.mH) - 2.0 * (Gb @ ih)
            gX = torch.cat([gU, gV], dim=-2)
        else:
            gX = gU
        if wide:
            gX = gX.mT
        prod = gX.conj() * Wd if gX.is_complex() else gX * Wd
        if per_matrix:
            D = prod.real.sum(dim=(-2, -1), keepdim=True) if prod.is_complex() else prod.sum(dim=(-2, -1), keepdim=True)
        else:
            D = prod.real.sum() if prod.is_complex() else prod.sum()
        a = alpha.reshape(n.shape)
        gW = s * gX - (a * D / (n * n * n)) * Wd
        galpha = (D / n).reshape(alpha.shape)
        return gW, galpha, None


def _dense_prep(W: torch.Tensor, alpha: torch.Tensor, M: Optional[torch.Tensor] = None):
    """Forward up to the Cayley system: norms, G = V'^T V' (GEMM), M = I + s (U' - U'^T) + s^2 G
    (k_dense_prep).  ``M``: optional [b, k, k] output buffer (a slice of a batched system)."""
    from . import ops, _lib as L
    Wb = W.detach().reshape(-1, W.shape[-2], W.shape[-1]).contiguous()
    al = alpha.detach().reshape(-1).contiguous().float()
    b, cout, cin = Wb.shape
    wide = cin > cout
    k = cout if wide else cin
    cfg = L.DenseConfig(b, cout, cin)
    lib, st = L.lib(), ops._stream(W.device)
    if not DENSE_NORM_PARTIALS:
        nrm = torch.linalg.vector_norm(Wb, dim=(-2, -1)).contiguous()
    else:
        # ||W|| as 256 partial sums per matrix ahead of the G GEMM, finished by the prep kernel (no
        # torch reduction on the map's forward chain)
        part = torch.empty(lib.fiode_dense_norm_workspace_bytes(ct.byref(cfg)) // 4, dtype=torch.float32,
                           device=W.device)
        L.check(lib.fiode_dense_norm_partials(st, ct.byref(cfg), Wb.data_ptr(), part.data_ptr(), part.numel() * 4),
                "fiode_dense_norm_partials")
    Vp = (Wb[:, :, k:].mT if wide else Wb[:, k:, :]) if max(cout, cin) > k else None
    G = ops.mm(Vp.mT, Vp, site="dense_fwd") if Vp is not None else None
    if M is None:
        M = torch.empty((b, k, k), dtype=torch.float32, device=W.device)
    if not DENSE_NORM_PARTIALS:
        L.check(lib.fiode_dense_cayley_prep(st, ct.byref(cfg), Wb.data_ptr(), al.data_ptr(), nrm.data_ptr(),
                                            ops._ptr(G), M.data_ptr()), "fiode_dense_cayley_prep")
    else:
        nrm = torch.empty(b, dtype=torch.float32, device=W.device)
        L.check(lib.fiode_dense_cayley_prep_normed(st, ct.byref(cfg), Wb.data_ptr(), al.data_ptr(), part.data_ptr(),
                                                   nrm.data_ptr(), ops._ptr(G), M.data_ptr()),
                "fiode_dense_cayley_prep_normed")
    return dict(Wb=Wb, al=al, nrm=nrm, wide=wide, k=k, Vp=Vp, cfg=cfg), M


def _dense_finish(st: dict, inv: torch.Tensor) -> torch.Tensor:
    """Q = [2 inv - I ; -2 s V' inv] in W's layout (P GEMM + k_dense_finish)."""
    from . import ops, _lib as L
    Wb, k = st["Wb"], st["k"]
    P = None                    # V' inv in W's layout (wide: its transpose inv^T V'^T = inv^T W[:, k:])
    if st["Vp"] is not None:
        P = (ops.mm(inv.mT, Wb[:, :, k:], site="dense_fwd") if st["wide"] else
             ops.mm(st["Vp"], inv, site="dense_fwd"))
    Q = torch.empty_like(Wb)
    L.check(L.lib().fiode_dense_cayley_finish(ops._stream(Wb.device), ct.byref(st["cfg"]), st["al"].data_ptr(),
                                              st["nrm"].data_ptr(), inv.data_ptr(), ops._ptr(P), Q.data_ptr()),
            "fiode_dense_cayley_finish")
    return Q


def _dense_backward(Wb, al, nrm, inv, gQ, wshape, ashape):
    """dL/dW, dL/dalpha of the dense Cayley map from dL/dQ (GEMMs + dense.hip stages)."""
    from . import ops, _lib as L
    b, cout, cin = Wb.shape
    wide = cin > cout
    k = cout if wide else cin
    R = max(cout, cin)
    gQb = gQ.reshape(b, cout, cin).contiguous()
    cfg = L.DenseConfig(b, cout, cin)
    lib, st = L.lib(), ops._stream(Wb.device)
    Vp = Gb = A = P2 = None
    if R > k:
        Vp = Wb[:, :, k:].mT if wide else Wb[:, k:, :]
        Gb = gQb[:, :, k:].mT if wide else gQb[:, k:, :]
        # A = V'^T Gb and P2 = Gb inv^T (W layout; wide: inv gQ[:, k:]) need only the inputs: one launch
        # for both (fiode_gemm_pair), so P2 leaves the A -> Ginv -> GMn -> H -> P1 chain
        A, P2 = (ops.mm_pair(Vp.mT, Gb, inv, gQb[:, :, k:], site="dense_bwd") if wide else
                 ops.mm_pair(Vp.mT, Gb, Gb, inv.mT, site="dense_bwd"))
    Ginv = torch.empty((b, k, k), dtype=torch.float32, device=Wb.device)
    L.check(lib.fiode_dense_cayley_ginv(st, ct.byref(cfg), al.data_ptr(), nrm.data_ptr(), gQb.data_ptr(),
                                        ops._ptr(A), Ginv.data_ptr()), "fiode_dense_cayley_ginv")
    ih = inv.mT
    if DENSE_GEMM and k % 64 == 0 and inv.is_contiguous() and inv.data_ptr() % 16 == 0 and Ginv.data_ptr() % 16 == 0:
        # GMn = inv^T (Ginv inv^T) by fiode_dense_gemm (256 workgroups at k = 512; the library's
        # 128 x 128 tiles leave 240 CUs idle on this latency-bound chain)
        T = torch.empty((b, k, k), dtype=torch.float32, device=Wb.device)
        GMn = torch.empty_like(T)
        L.check(lib.fiode_dense_gemm(st, b, k, 0, 1, Ginv.data_ptr(), inv.data_ptr(), T.data_ptr()), "fiode_dense_gemm")
        L.check(lib.fiode_dense_gemm(st, b, k, 1, 0, inv.data_ptr(), T.data_ptr(), GMn.data_ptr()), "fiode_dense_gemm")
    else:
        GMn = ops.mm(ih, ops.mm(Ginv, ih, site="dense_bwd"), site="dense_bwd")
    gX = torch.empty_like(Wb)                    # W layout
    H = torch.empty((b, k, k), dtype=torch.float32, device=Wb.device)
    L.check(lib.fiode_dense_cayley_h(st, ct.byref(cfg), GMn.data_ptr(), gX.data_ptr(), H.data_ptr()),
            "fiode_dense_cayley_h")
    P1 = None                       # V' H in W's layout (wide: H^T W[:, k:])
    if R > k:
        P1 = ops.mm(H.mT, Wb[:, :, k:], site="dense_bwd") if wide else ops.mm(Vp, H, site="dense_bwd")
    gW = torch.empty_like(Wb)
    ga = torch.empty(b, dtype=torch.float32, device=Wb.device)
    ws = torch.empty(max(1, lib.fiode_dense_cayley_workspace_bytes(ct.byref(cfg))), dtype=torch.uint8,
                     device=Wb.device)
    L.check(lib.fiode_dense_cayley_grad(st, ct.byref(cfg), Wb.data_ptr(), al.data_ptr(), nrm.data_ptr(),
                                        ops._ptr(P1), ops._ptr(P2), gX.data_ptr(), gW.data_ptr(), ga.data_ptr(),
                                        ws.data_ptr(), ws.numel()), "fiode_dense_cayley_grad")
    return gW.reshape(wshape), ga.reshape(ashape)


def _dense_fused_ok(W: torch.Tensor) -> bool:
    from . import _lib as L
    k = min(W.shape[-2], W.shape[-1])
    lib = L.lib()
    return (DENSE_FUSED_INVERSE and W.is_cuda and hasattr(lib, "fiode_dense_cayley_inverse")
            and lib.fiode_dense_inverse_flag_bytes(k) > 0)


def _dense_forward_fused(W: torch.Tensor, alpha: torch.Tensor):
    """The map forward with the one-launch inverse building M on load (fiode_dense_cayley_inverse):
    norm partials (+ the inverse's flag words zeroed in the same launch), [G GEMM], the inverse (+ Q
    for a square map), [P GEMM + k_dense_finish].  The same M, inverse and Q as _dense_prep ->
    _block_inverse -> _dense_finish, bit for bit (dense.hip k_dense_prep's arithmetic on load)."""
    from . import ops, _lib as L
    Wb = W.detach().reshape(-1, W.shape[-2], W.shape[-1]).contiguous()
    al = alpha.detach().reshape(-1).contiguous().float()
    b, cout, cin = Wb.shape
    wide = cin > cout
    k = cout if wide else cin
    cfg = L.DenseConfig(b, cout, cin)
    lib, stream = L.lib(), ops._stream(W.device)
    per = lib.fiode_block_inverse_workspace_bytes(k)
    ws = ops._Workspace.get(W.device, b * per, f"denseinv{torch.cuda.current_stream(W.device).cuda_stream}")
    part = torch.empty(lib.fiode_dense_norm_workspace_bytes(ct.byref(cfg)) // 4, dtype=torch.float32, device=W.device)
    L.check(lib.fiode_dense_norm_partials_clear(stream, ct.byref(cfg), Wb.data_ptr(), part.data_ptr(), part.numel() * 4,
                                                ws.data_ptr(), lib.fiode_dense_inverse_flag_bytes(k) // 4, per),
            "fiode_dense_norm_partials_clear")
    Vp = (Wb[:, :, k:].mT if wide else Wb[:, k:, :]) if max(cout, cin) > k else None
    G = ops.mm(Vp.mT, Vp, site="dense_fwd") if Vp is not None else None
    nrm = torch.empty(b, dtype=torch.float32, device=W.device)
    inv = torch.empty((b, k, k), dtype=torch.float32, device=W.device)
    Q = torch.empty_like(Wb) if Vp is None else None
    L.check(lib.fiode_dense_cayley_inverse(stream, ct.byref(cfg), Wb.data_ptr(), al.data_ptr(), part.data_ptr(),
                                           ops._ptr(G), nrm.data_ptr(), inv.data_ptr(), ops._ptr(Q), ws.data_ptr(),
                                           ws.numel()), "fiode_dense_cayley_inverse")
    st = dict(Wb=Wb, al=al, nrm=nrm, wide=wide, k=k, Vp=Vp, cfg=cfg)
    if Q is None:
        Q = _dense_finish(st, inv)
    return st, inv, Q


class _DenseCayleyFn(torch.autograd.Function):
    """cayley(alpha W / ||W||) for a batch of real [cout, cin] matrices (per-matrix norm and alpha):
    the same forward / analytic backward as _CayleyScaledFn, with the GEMMs as library GEMMs and
    every elementwise stage between them one HIP kernel (fiode_dense_cayley_*; dense.hip).  For
    k = min(cout, cin) = 128 .. 512 (the backbone's 512 maps, the dynamics' 128 x 128) the inverse is
    one launch that builds M on load (_dense_forward_fused): 2 launches for a square map's forward,
    5 for a wide one (norm partials, G GEMM, inverse, P GEMM, finish)."""

    @staticmethod
    def forward(ctx, W, alpha):
        if _dense_fused_ok(W):
            st, inv, Q = _dense_forward_fused(W, alpha)
        else:
            st, M = _dense_prep(W, alpha)
            inv = _block_inverse(M)
            Q = _dense_finish(st, inv)
        ctx.save_for_backward(st["Wb"], st["al"], st["nrm"], inv)
        ctx.shapes = (W.shape, alpha.shape)
        ctx.step_stream = STEP_STREAM
        return Q.reshape(W.shape)

    @staticmethod
    def backward(ctx, gQ):
        Wb, al, nrm, inv = ctx.saved_tensors
        return _run_on_step_stream(DENSE_BWD_ON_MAIN, ctx.step_stream,
                                   lambda: _dense_backward(Wb, al, nrm, inv, gQ, *ctx.shapes))


class _SmallCayleyFn(torch.autograd.Function):
    """cayley(alpha W / ||W||) for a batch of real [cout, cin] matrices with k = min(cout, cin)
    <= 16: forward and backward are one kernel each (fiode_small_cayley_*; small_cayley.hip) --
    the same formula as _CayleyScaledFn, one workgroup per matrix."""

    @staticmethod
    def forward(ctx, W, alpha):
        from . import ops, _lib as L
        Wb = W.detach().reshape(-1, W.shape[-2], W.shape[-1]).contiguous()
        al = alpha.detach().reshape(-1).contiguous().float()
        b, cout, cin = Wb.shape
        k = min(cout, cin)
        Q = torch.empty_like(Wb)
        inv = torch.empty((b, k, k), dtype=torch.float32, device=W.device)
        nrm = torch.empty(b, dtype=torch.float32, device=W.device)
        L.check(L.lib().fiode_small_cayley_forward(ops._stream(W.device), b, cout, cin, Wb.data_ptr(), al.data_ptr(),
                                                   Q.data_ptr(), inv.data_ptr(), nrm.data_ptr()),
                "fiode_small_cayley_forward")
        ctx.save_for_backward(Wb, al, nrm, inv)
        ctx.shapes = (W.shape, alpha.shape)
        ctx.step_stream = STEP_STREAM
        return Q.reshape(W.shape)

    @staticmethod
    def backward(ctx, gQ):
        return _run_on_step_stream(SMALL_BWD_ON_MAIN, ctx.step_stream, lambda: _SmallCayleyFn._backward(ctx, gQ))

    @staticmethod
    def _backward(ctx, gQ):
        from . import ops, _lib as L
        Wb, al, nrm, inv = ctx.saved_tensors
        wshape, ashape = ctx.shapes
        b, cout, cin = Wb.shape
        gQb = gQ.reshape(b, cout, cin).contiguous().float()
        gW = torch.empty_like(Wb)
        ga = torch.empty(b, dtype=torch.float32, device=Wb.device)
        L.check(L.lib().fiode_small_cayley_backward(ops._stream(Wb.device), b, cout, cin, Wb.data_ptr(), al.data_ptr(),
                                                    nrm.data_ptr(), inv.data_ptr(), gQb.data_ptr(), gW.data_ptr(),
                                                    ga.data_ptr()), "fiode_small_cayley_backward")
        return gW.reshape(wshape), ga.reshape(ashape)


def _small_ok(W: torch.Tensor) -> bool:
    from . import _lib as L
    cout, cin = W.shape[-2], W.shape[-1]
    k, R = min(cout, cin), max(cout, cin)
    return k <= L.FIODE_SMALL_CAYLEY_MAX_K and R * k <= L.FIODE_SMALL_CAYLEY_MAX_RK


def cayley_scaled(W: torch.Tensor, alpha: torch.Tensor, per_matrix: bool = False) -> torch.Tensor:
    """cayley(alpha * W / ||W||) (convert_cayley's parametrisation, classification.py:282-293).
    Real matrices on ROCm (one matrix, or a batch with per-matrix norms) take one kernel per
    direction when k = min(cout, cin) <= 16 (_SmallCayleyFn), else the fused stages of
    _DenseCayleyFn; complex ones and a batch under one norm take _CayleyScaledFn."""
    if W.is_cuda and W.dtype == torch.float32 and (W.dim() == 2 or per_matrix) and DENSE_FUSED:
        if SMALL_FUSED and _small_ok(W):
            return _SmallCayleyFn.apply(W, alpha)
        return _DenseCayleyFn.apply(W, alpha)
    return _CayleyScaledFn.apply(W, alpha, per_matrix)


DENSE_FUSED = True
SMALL_FUSED = True
DENSE_FUSED_INVERSE = True   # the one-launch inverse builds M itself (tests compare it with the staged path)


def cayley(W: torch.Tensor) -> torch.Tensor:
    """Orthogonal (or orthonormal-column) matrix from an unconstrained W [.., cout, cin]:
    with U = W[:cin], V = W[cin:], A = U - U^H + V^H V:
        Q = [(I+A)^-1 (I-A); -2 V (I+A)^-1] = [2 (I+A)^-1 - I; -2 V (I+A)^-1].
    Wide matrices (cin > cout) are handled through the transpose."""
    if W.dim() == 2:
        return cayley(W.unsqueeze(0)).squeeze(0)
    cout, cin = W.shape[-2], W.shape[-1]
    if cin > cout:
        return cayley(W.transpose(-2, -1)).transpose(-2, -1)
    U, V = W[..., :cin, :], W[..., cin:, :]
    eye = torch.eye(cin, dtype=W.dtype, device=W.device)
    A = U - U.mH
    if cout > cin:
        A = A + V.mH @ V
    inv = _CayleyInverse.apply(eye + A)
    top = 2.0 * inv - eye
    if cout == cin:
        return top
    return torch.cat([top, -2.0 * (V @ inv)], dim=-2)


# Backward placement of the prefetched maps.  autograd runs a node's backward on the stream its
# forward ran on (a side stream); with these flags the backward of the spectral / dense maps runs
# on the stream the step was launched from instead: STEP_STREAM is set by
# LyapunovLearning.compute_loss only while it runs (step_stream_scope) and each map records it on
# its autograd ctx at forward time, so a later eager or non-parallel step never sends work to a
# stale (e.g. graph-capture) stream.  The hipGraph executor places that stream on another
# hardware queue.  With the executor on 2 internal
# streams (bench.py) the dense maps' backward on the step stream measured 2.28 -> 2.24 ms per step
# in the interleaved A/B (tools/ab_step.py); the spectral maps' is slower there (2.35 ms).
SPECTRAL_BWD_ON_MAIN = False
DENSE_BWD_ON_MAIN = True
DENSE_GEMM = True          # GMn by fiode_dense_gemm (tools/ab_step.py `lib_gmn` measures the library form)
DENSE_NORM_PARTIALS = True  # ||W|| by fiode_dense_norm_partials + the prep kernel (`torch_norm`: vector_norm)
SMALL_BWD_ON_MAIN = False
STEP_STREAM: Optional[torch.cuda.Stream] = None


class step_stream_scope:
    """Context manager: STEP_STREAM = ``stream`` inside, the previous value restored on exit."""

    def __init__(self, stream):
        self.stream = stream

    def __enter__(self):
        global STEP_STREAM
        self.prev, STEP_STREAM = STEP_STREAM, self.stream
        return self

    def __exit__(self, *exc):
        global STEP_STREAM
        STEP_STREAM = self.prev
        return False


def _run_on_step_stream(flag: bool, step_stream, fn):
    tgt = step_stream if flag else None
    cur = torch.cuda.current_stream()
    if tgt is None or tgt == cur:
        return fn()
    tgt.wait_stream(cur)
    with torch.cuda.stream(tgt):
        out = fn()
    cur.wait_stream(tgt)
    for t in out:
        if isinstance(t, torch.Tensor):
            t.record_stream(cur)
    return out


def _prefetch(stream: torch.cuda.Stream, fn):
    """Run fn() on `stream` (forked from the current stream); returns (result, done event)."""
    main = torch.cuda.current_stream(stream.device)
    stream.wait_stream(main)
    with torch.cuda.stream(stream):
        out = fn()
        ev = torch.cuda.Event()
        ev.record(stream)
    return out, ev


def _take(pre):
    """Join a prefetched result into the current stream."""
    out, ev = pre
    main = torch.cuda.current_stream()
    main.wait_event(ev)
    for t in (out.values() if isinstance(out, dict) else (out,)):
        if isinstance(t, torch.Tensor):
            t.record_stream(main)
    return out


class CayleyLinear(nn.Linear):
    """nn.Linear whose effective weight is cayley(alpha * W / ||W||_F) (state_dict keys
    ``weight``, ``bias``, ``alpha``, as the reference's checkpoints carry)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__(in_features, out_features, bias)
        self.alpha = nn.Parameter(self.weight.detach().norm().reshape(1).clone())
        self._Q = None
        self._pre = None

    def reset_parameters(self) -> None:
        std = 1.0 / math.sqrt(self.weight.shape[1])
        nn.init.uniform_(self.weight, -std, std)
        if self.bias is not None:
            nn.init.uniform_(self.bias, -std, std)
        self._Q = None

    def effective_weight(self) -> torch.Tensor:
        return cayley_scaled(self.weight, self.alpha)

    def prefetch(self, stream: torch.cuda.Stream) -> None:
        """Compute this step's Cayley map on a side stream (its latency-bound inverse overlaps
        the layers before it); the next training forward joins it."""
        self._pre = _prefetch(stream, self.effective_weight)

    def forward_weight_unjoined(self):
        """(Q, done event or None): forward_weight, but a pending prefetched map is handed out
        WITHOUT making the current stream wait for it -- the caller waits on the event right before
        its first use of Q (the stream-order bookkeeping of _take is done here)."""
        if self._pre is not None and self.training:
            (Q, ev), self._pre = self._pre, None
            Q.record_stream(torch.cuda.current_stream(Q.device))
            self._Q = Q.detach()
            return Q, ev
        return self.forward_weight(), None

    def forward_weight(self) -> torch.Tensor:
        """The effective weight this forward uses (the prefetched map when one is pending)."""
        if self._pre is not None and self.training:
            Q = _take(self._pre)
            self._pre = None
        elif self.training or self._Q is None:
            Q = self.effective_weight()
        else:
            Q = self._Q
        # kept detached: a stored Q with its graph would keep the step's autograd nodes (and the
        # parameters' AccumulateGrad nodes) alive into the next step
        self._Q = Q.detach()
        return Q if self.training else self._Q

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return F.linear(x, self.forward_weight(), self.bias)


# KWLargeConcat's head (Linear -> GroupSort -> Linear -> GroupSort -> Linear) as one autograd node
# whose backward keeps only the input-gradient chain on the step's stream (see _LinearHeadFn)
HEAD_WGRAD_SIDE = os.environ.get("FIODE_HEAD_WGRAD_SIDE", "1") != "0"
_HEAD_STREAMS: dict = {}


# side streams of the head's weight gradients: 3 = one stream per layer (the step's stream joins
# them all at the end of the head's backward; layer 3's is also the conv weight gradients' stream).
# With 1 the three layers' products and bias sums ran in sequence on one stream, and that ~55 us
# chain, not the input-gradient chain, was the head backward's part of the step's dependency path
# (profiles/r06/dag_warm/): 3 streams measured 8-23 us faster per step, 2 streams or the bias sums on
# three more streams slower (profiles/r06/ab_head_wgrad_streams.json)
HEAD_WGRAD_STREAMS = int(os.environ.get("FIODE_HEAD_WGRAD_STREAMS", "3"))


def _head_stream(dev: torch.device, k: int = 0) -> torch.cuda.Stream:
    key = (dev.index, k % HEAD_WGRAD_STREAMS)
    if key not in _HEAD_STREAMS:
        _HEAD_STREAMS[key] = new_stream(dev)
    return _HEAD_STREAMS[key]


class _LinearHeadFn(torch.autograd.Function):
    """y = L3(gs(L2(gs(L1(h))))) with L_k(x) = x Q_k^T + b_k (F.linear's addmm) and gs the GroupSort
    kernel.  Autograd's addmm backward runs each layer's input gradient, weight gradient and bias
    sum in sequence on one stream, so the next layer's input gradient waited for the weight
    gradient it does not need (the head's backward is on the step's critical path).  Here the
    weight / bias gradients (the same GEMM g^T x and column sum) of every layer run on a side
    stream of their own (HEAD_WGRAD_STREAMS) forked as soon as that layer's output gradient exists,
    beside the input-gradient chain, and join the step's stream once at the end.  The products go through ops.mm (the library GEMM
    at this site: ops.MM_LIBRARY_SITES), the output layer fiode_head_out / _backward_gs when it has
    <= 16 outputs (KWLargeConcat's 10 classes; a wider out_dim, e.g. make_ortho_KWLarge_Concat's
    default 128, takes ops.mm + the GroupSort kernel)."""

    @staticmethod
    def forward(ctx, h, Q1, b1, Q2, b2, Q3, b3, joins=None):
        from . import ops
        # joins: the done events of Q2 / Q3 still being computed on their prefetch streams, waited
        # for right before the layer that reads them (the first layer runs meanwhile)
        j2, j3 = joins if joins is not None else (None, None)
        cur = torch.cuda.current_stream(h.device)
        y1 = ops.mm(h, Q1.t(), bias=b1, site="head")
        z1 = ops.groupsort_forward(y1, 1)
        if j2 is not None:
            cur.wait_event(j2)
        y2 = ops.mm(z1, Q2.t(), bias=b2, site="head")
        z2 = ops.groupsort_forward(y2, 1)
        if j3 is not None:
            cur.wait_event(j3)
        out_k = _head_out_ok(Q3)
        # the 512 -> 10 output layer: the library ran it on one workgroup (~15 us on the chain)
        out = ops.head_out(z2, Q3, b3) if out_k else ops.mm(z2, Q3.t(), bias=b3, site="head")
        ctx.save_for_backward(h, Q1, Q2, Q3, y1, z1, y2, z2)
        ctx.out_k = out_k
        return out

    @staticmethod
    def backward(ctx, g):
        from . import ops
        h, Q1, Q2, Q3, y1, z1, y2, z2 = ctx.saved_tensors
        g = g.contiguous()
        cur = torch.cuda.current_stream(g.device)
        sides = []
        wg = {}

        def wgrad(k, gk, x):
            side = _head_stream(g.device, k)
            if side not in sides:
                sides.append(side)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                wg[k] = (ops.mm(gk.t(), x, site="head"), gk.sum(0))
            gk.record_stream(side)
            x.record_stream(side)

        wgrad(3, g, z2)
        g2 = ops.head_out_backward_gs(g, Q3, y2) if ctx.out_k else ops.groupsort_backward(y2, ops.mm(g, Q3, site="head"), 1)
        wgrad(2, g2, z1)
        g1 = ops.groupsort_backward(y1, ops.mm(g2, Q2, site="head"), 1)
        wgrad(1, g1, h)
        dh = ops.mm(g1, Q1, site="head")
        for side in sides:
            cur.wait_stream(side)
        for dW, db in wg.values():
            dW.record_stream(cur)
            db.record_stream(cur)
        return dh, wg[1][0], wg[1][1], wg[2][0], wg[2][1], wg[3][0], wg[3][1], None


# the head's output layer and its GroupSort input gradient by fiode_head_out / _backward_gs (<= 16
# outputs: HEAD_JMAX of backbone.hip)
HEAD_OUT_KERNEL = True
HEAD_OUT_MAX_J = 16


def _head_out_ok(Q3: torch.Tensor) -> bool:
    return HEAD_OUT_KERNEL and Q3.shape[0] <= HEAD_OUT_MAX_J


def linear_head(mods, h: torch.Tensor):
    """Apply KWLargeConcat's head modules to h: one _LinearHeadFn node when training on ROCm with
    the GroupSort head, else module by module."""
    fusable = (HEAD_WGRAD_SIDE and h.is_cuda and len(mods) == 5 and
               all(isinstance(m, CayleyLinear) and m.training and m.bias is not None for m in mods[0::2]) and
               all(isinstance(m, GroupSort) for m in mods[1::2]) and torch.is_grad_enabled())
    if not fusable:
        for m in mods:
            h = m(h)
        return h
    l1, l2, l3 = mods[0::2]
    Q1 = l1.forward_weight()
    if HEAD_LATE_JOIN:
        (Q2, j2), (Q3, j3) = l2.forward_weight_unjoined(), l3.forward_weight_unjoined()
        return _LinearHeadFn.apply(h.contiguous(), Q1, l1.bias, Q2, l2.bias, Q3, l3.bias, (j2, j3))
    return _LinearHeadFn.apply(h.contiguous(), Q1, l1.bias, l2.forward_weight(), l2.bias,
                               l3.forward_weight(), l3.bias)


# the head joins the 512 -> 512 and 512 -> 10 maps' prefetch right before the layer that reads them,
# not before its first layer (tools/ab_step.py `head_join_early`)
HEAD_LATE_JOIN = True



class _GroupSortFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cdim: int):
        from . import ops
        y = ops.groupsort_forward(x, cdim)
        ctx.save_for_backward(x)
        ctx.cdim = cdim
        return y

    @staticmethod
    def backward(ctx, g):
        from . import ops
        x, = ctx.saved_tensors
        return ops.groupsort_backward(x, g, ctx.cdim), None


class GroupSort(nn.Module):
    """Sort pairs of channel halves: [max(a, b), min(a, b)] along the channel dim (1, or
    ``channel_dim`` for the spatial-major conv stack).  On ROCm tensors one HIP kernel each way
    (fiode_groupsort_*; ties split the gradient like torch.maximum); host tensors take the torch
    ops."""

    def __init__(self, channel_dim: int = 1):
        super().__init__()
        self.channel_dim = channel_dim

    def forward(self, x: torch.Tensor, channel_dim: Optional[int] = None) -> torch.Tensor:
        cd = self.channel_dim if channel_dim is None else channel_dim
        if x.is_cuda:
            return _GroupSortFn.apply(x, cd)
        a, b = x.split(x.size(cd) // 2, cd)
        return torch.cat([torch.maximum(a, b), torch.minimum(a, b)], dim=cd)


class _SpectralCayleyFn(torch.autograd.Function):
    """Q[f] = cayley(alpha Wf[f] / ||Wf||) for all rFFT frequencies of a 3x3 CayleyConv in two
    fused launches each way (fiode_spectral_cayley_*; spectral.hip) instead of the ~75 kernels of
    rfft2 + shift + conj + cayley_scaled and their autograd."""

    @staticmethod
    def forward(ctx, weight, alpha, n: int):
        from . import ops
        Q, inv, ws = ops.spectral_cayley_forward(weight.detach(), alpha.detach(), n)
        ctx.save_for_backward(weight, alpha, inv, ws)
        ctx.n = n
        ctx.step_stream = STEP_STREAM
        return Q

    @staticmethod
    def backward(ctx, gQ):
        from . import ops
        weight, alpha, inv, ws = ctx.saved_tensors
        gw, ga = _run_on_step_stream(SPECTRAL_BWD_ON_MAIN, ctx.step_stream, lambda: ops.spectral_cayley_backward(
            gQ.contiguous(), weight.detach(), alpha.detach(), ctx.n, inv, ws))
        return gw, ga.reshape(alpha.shape), None


class _SpectralCayleyStoredFn(torch.autograd.Function):
    """The Q of a CayleyConv whose map was computed AHEAD, into fixed buffers (CayleyConv
    pipeline_on / refresh_map: at the end of the previous training step, right after this layer's
    parameters were updated): forward hands out the stored Q (no kernel); backward is
    _SpectralCayleyFn's, from the stored inverse and workspace, then ``store["on_grads"]`` (if set)
    gets (dL/dweight, dL/dalpha) -- GraphTrainStep updates the layer's parameters there and
    computes its next map while the rest of the backward runs."""

    @staticmethod
    def forward(ctx, weight, alpha, n: int, store: dict):
        ctx.save_for_backward(weight, alpha)
        ctx.store, ctx.n = store, n
        return store["Q"].detach()

    @staticmethod
    def backward(ctx, gQ):
        from . import ops
        weight, alpha = ctx.saved_tensors
        st = ctx.store
        gw, ga = ops.spectral_cayley_backward(gQ.contiguous(), weight.detach(), alpha.detach(), ctx.n, st["inv"],
                                              st["ws"])
        ga = ga.reshape(alpha.shape)
        hook = st.get("on_grads")
        if hook is not None:
            hook(gw, ga)
        return gw, ga, None, None


class _SpectralConvFn(torch.autograd.Function):
    """y = [GroupSort](irfft2(Q[f] @ rfft2(x)[f]) + bias) on spatial-major activations, the
    transforms as HIP kernels that read / write the GEMM layout [f][C][B] (sconv.hip), the
    per-frequency channel products as batched complex GEMMs.  Backward (torch's conventions for
    the real transforms, w_kb = 1 at kb = 0, n/2 and 2 between):
        G = rfft2(d/dpre),  dQ = (w_kb / n^2) G X^H,  dx = irfft2(Q^H G),  dbias = sum_b Re G[0]."""

    @staticmethod
    def forward(ctx, x, Q, bias, n: int, downsample: bool, groupsort: bool, norm=None, nchw_out: bool = False):
        from . import ops
        nf, cout, cin = Q.shape
        if norm is not None:     # x: the NCHW network input, normalised on load (no input gradient)
            B = x.shape[0]
            X = ops.sconv_rfft2_nchw(x.detach(), norm[0], norm[1], n)
        else:
            B = x.shape[-1]
            X = ops.sconv_rfft2(x.detach(), n, cin, B, downsample=downsample)
        bd = None if bias is None else bias.detach()
        if cin <= SCONV_QX_MAX_K and not downsample:
            # few input channels (conv 1: 3): the product formed in the inverse transform's loads
            y, code = ops.sconv_irfft2_qx(Q.detach(), X, n, B, bias=bd, groupsort=groupsort, nchw=nchw_out)
        else:
            y, code = ops.sconv_irfft2(ops.cgemm(Q.detach(), X), n, cout, B, bias=bd, groupsort=groupsort,
                                       nchw=nchw_out)
        ctx.save_for_backward(X, Q, code)
        ctx.cfg = (n, downsample, groupsort, bias is not None, cin, cout, B)
        ctx.nchw_out = nchw_out
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import ops
        X, Q, code = ctx.saved_tensors
        n, downsample, groupsort, has_bias, cin, cout, B = ctx.cfg
        gy = gy.contiguous()
        if groupsort:
            G = ops.sconv_rfft2(None, n, cout, B, gy=gy, code=code, nchw=ctx.nchw_out)
        else:
            G = ops.sconv_rfft2(gy, n, cout, B)
        gx = gQ = gb = None
        need_x, need_q, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], has_bias and ctx.needs_input_grad[2]
        wq = None
        if need_q:
            key = (n, str(G.device))
            wq = _SPECTRAL_GRAD_WEIGHTS.get(key)
            if wq is None:
                kb = torch.arange(n // 2 + 1, device=G.device)
                w = torch.where((kb == 0) | (kb == n // 2), 1.0, 2.0) / float(n * n)
                wq = _SPECTRAL_GRAD_WEIGHTS[key] = w.repeat(n).reshape(-1, 1, 1)

        def wgrad():        # dL/dQ = w G X^H: fiode_cgemm with B = X^H read from X and w folded in
            if need_q and CONV_WGRAD_LIB:          # (the library GEMM: note at CONV_WGRAD_LIB)
                gq = torch.matmul(G, X.mH) * wq
            else:
                gq = ops.cgemm(G, X, conj_trans_b=True, scale=wq.reshape(-1)) if need_q else None
            gbias = G[0].real.sum(-1) if need_b else None
            return gq, gbias
        # the weight / bias gradients beside the input gradient (which alone is on the backward's
        # critical chain), on the side stream of the linear head's, joined before returning
        side = _head_stream(G.device) if (CONV_WGRAD_SIDE and G.is_cuda and need_x and (need_q or need_b)) else None
        if side is not None:
            cur = torch.cuda.current_stream(G.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                gQ, gb = wgrad()
            G.record_stream(side)
            X.record_stream(side)
        if need_x:
            gx, _ = ops.sconv_irfft2(_q_h_g(Q, G), n, cin, B, downsample=downsample)
        if side is not None:
            cur.wait_stream(side)
            for t in (gQ, gb):
                if t is not None:
                    t.record_stream(cur)
        else:
            gQ, gb = wgrad()
        return gx, gQ, gb, None, None, None, None, None


_SPECTRAL_GRAD_WEIGHTS = {}
# The per-frequency channel products Q X and Q^H G are fiode_cgemm (cgemm.hip), not torch.matmul (the
# library's batched complex GEMM: one 128 x 64 tile per frequency; the n = 8 layer's forward 41 -> 16
# us, conv 3's input gradient 16 -> 10, conv 1's forward 13 -> 10 us; step -25 to -40 us in the
# alternating A/B, profiles/r05bd).  The weight gradient w G X^H on the side stream stays the library
# GEMM + the scale: the one fiode_cgemm launch (conjugate-transposed B, w folded in) measured 4.6 us
# slower in the step (profiles/r06/ab_gemm_sites.json; round 5: 10-20 us, profiles/r05bj).
# CONV_WGRAD_LIB = False takes the fiode_cgemm launch.
CONV_WGRAD_LIB = True
# conv layers with at most this many input channels (conv 1: 3) form Q X inside the inverse
# transform's loads (fiode_sconv_irfft2_qx; the kernel's limit is 4): no GEMM launch, no [f][C][B]
# product in HBM
SCONV_QX_MAX_K = 4


def _q_h_g(Q, G):
    from . import ops
    return ops.cgemm(Q.detach(), G, conj_trans_a=True)


CONV_WGRAD_SIDE = os.environ.get("FIODE_CONV_WGRAD_SIDE", "1") != "0"


# The conv layers' map-ahead work (map backward, early update, refresh) runs on one stream per layer.
# (Their weight gradients on those streams instead of the head's side stream -- no join: 110-140 us
# SLOWER in the step, profiles/r05an -- and one stream shared by all layers were measured and removed.)
def _conv_map_stream(device) -> "torch.cuda.Stream":
    return new_stream(device)


class CayleyConv(nn.Conv2d):
    """Orthogonal circular convolution parametrised per frequency: for each of the n*(n/2+1)
    rFFT frequencies the cout x cin channel matrix is Cayley-mapped, y = irfft2(Q(w) xfft).
    stride=2 is an invertible 2x2 space-to-channel downsample followed by a stride-1 conv on
    4*cin channels (the public design's StridedConv)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, bias: bool = True):
        self.downsample = stride == 2
        super().__init__(in_channels * (4 if self.downsample else 1), out_channels, kernel_size, stride=1,
                         padding=kernel_size // 2, bias=bias)
        self.alpha = nn.Parameter(torch.ones(1))
        self._alpha_init = False
        self.fused = True               # fused spectral Cayley kernels on ROCm (spectral.hip)
        self._fused_shapes = {}
        self._shift = {}
        self._n = None
        self._pre = None
        self._store = None              # map computed ahead (pipeline_on), else None

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self._alpha_init = True          # a loaded alpha is kept (no data-dependent re-init)

    def _shift_matrix(self, n: int, device) -> torch.Tensor:
        key = (n, str(device))
        if key not in self._shift:
            s = -((self.weight.shape[2] - 1) // 2)
            k = torch.arange(n, device=device, dtype=torch.float64)
            grid = k[None, :] + k[:, None]
            sh = torch.exp(2j * math.pi * s * grid / n)[:, : n // 2 + 1]
            self._shift[key] = sh.reshape(n * (n // 2 + 1), 1, 1).to(torch.complex64)
        return self._shift[key]

    def spectral_weight(self, n: int, device) -> torch.Tensor:
        """The per-frequency orthogonal channel matrices Q [n (n/2+1), cout, cin] for n x n inputs.
        ROCm tensors of a supported shape (3x3 taps, min(cout, cin) <= 64) take the fused HIP map
        (_SpectralCayleyFn); otherwise the op-by-op formula below (also the tests' reference)."""
        if self.fused and self._alpha_init and self.weight.is_cuda and self._fused_ok(n):
            return _SpectralCayleyFn.apply(self.weight, self.alpha, n)
        return self.spectral_weight_reference(n, device)

    def _fused_ok(self, n: int) -> bool:
        ok = self._fused_shapes.get(n)
        if ok is None:
            from . import ops
            ok = self._fused_shapes[n] = ops.spectral_supported(tuple(self.weight.shape), n)
        return ok

    def spectral_weight_reference(self, n: int, device) -> torch.Tensor:
        """rfft2 of the taps, the shift of the 'same' padding, conj, cayley_scaled (PyTorch ops)."""
        cout, cin = self.weight.shape[:2]
        nf = n * (n // 2 + 1)
        wf = torch.fft.rfft2(self.weight, (n, n)).reshape(cout, cin, nf).permute(2, 0, 1).conj()
        wf = self._shift_matrix(n, device) * wf
        if not self._alpha_init:
            with torch.no_grad():
                self.alpha.fill_(float(wf.norm()))
            self._alpha_init = True
        return cayley_scaled(wf, self.alpha)

    # ---- maps computed ahead (GraphTrainStep): the next step's Q right after this step's update --
    def pipeline_on(self) -> bool:
        """Keep this layer's map in fixed buffers, computed ahead by refresh_map (now, from the
        current parameters).  Only for the fused map after one training forward (input size known);
        returns whether the layer is pipelined."""
        if not (self.fused and self._alpha_init and self._n is not None and self.weight.is_cuda
                and self._fused_ok(self._n)):
            return False
        from . import ops
        Q, inv, ws = ops.spectral_cayley_forward(self.weight.detach(), self.alpha.detach(), self._n)
        self._store = {"Q": Q, "inv": inv, "ws": ws, "n": self._n, "stream": _conv_map_stream(self.weight.device)}
        return True

    def pipeline_off(self) -> None:
        self._store = None

    def refresh_map(self) -> None:
        """Recompute the stored map from the current parameters (same kernels as the step-start
        map, so the same Q bit for bit), on the current stream."""
        from . import ops
        st = self._store
        ops.spectral_cayley_forward(self.weight.detach(), self.alpha.detach(), st["n"],
                                    out=(st["Q"], st["inv"], st["ws"]))

    def prefetch(self, stream: torch.cuda.Stream) -> None:
        """Compute this step's spectral Cayley maps on a side stream (needs one forward first, to
        know the input size and initialise alpha)."""
        if self._store is not None:
            return
        if self._n is not None and self._alpha_init:
            n = self._n
            self._pre = _prefetch(stream, lambda: self.spectral_weight(n, self.weight.device))

    def _take_spectral(self, n: int, device) -> torch.Tensor:
        st = self._store
        if st is not None and self.training and st["n"] == n and torch.is_grad_enabled():
            # the node's backward (map backward + the store's hook) runs on the layer's own stream
            side = st["stream"]
            main = torch.cuda.current_stream(device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                Q = _SpectralCayleyStoredFn.apply(self.weight, self.alpha, n, st)
            main.wait_stream(side)
            self._pre = None
            return Q
        if self._pre is not None and self.training and self._n == n:
            Q = _take(self._pre)
        else:
            Q = self.spectral_weight(n, device)
        self._pre = None
        self._n = n
        return Q

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.downsample:
            b, c, h, w = x.shape
            x = x.reshape(b, c, h // 2, 2, w // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(b, c * 4, h // 2, w // 2)
        cout, cin = self.weight.shape[:2]
        B, _, n, _ = x.shape
        nf = n * (n // 2 + 1)
        xf = torch.fft.rfft2(x).permute(2, 3, 1, 0).reshape(nf, cin, B)
        Q = self._take_spectral(n, x.device)
        yf = (Q @ xf).reshape(n, n // 2 + 1, cout, B)
        y = torch.fft.irfft2(yf.permute(3, 2, 0, 1), s=(n, n))
        if self.bias is not None:
            y = y + self.bias[:, None, None]
        return y

    def forward_hwcb_fused(self, x: torch.Tensor, groupsort: bool, nchw_out: bool = False) -> torch.Tensor:
        """forward_hwcb (+ the following GroupSort) with the transforms as HIP kernels
        (_SpectralConvFn): [n][n][cin][B] (stride 2: [2n][2n][cin/4][B]) -> [n][n][cout][B], or with
        nchw_out (GroupSort only) [B][cout][n][n] -- the last conv, whose output the flatten reads."""
        n = x.shape[0] // 2 if self.downsample else x.shape[0]
        Q = self._take_spectral(n, x.device)
        return _SpectralConvFn.apply(x, Q, self.bias, n, self.downsample, groupsort, None,
                                     bool(nchw_out and groupsort))

    def forward_nchw_fused(self, x: torch.Tensor, mu: torch.Tensor, sd, groupsort: bool) -> torch.Tensor:
        """forward_hwcb_fused of the network's first layer straight from the NCHW input x [B][C][n][n]
        with the preceding Normalize's (x - mu) / sd applied in the transform's loads (one launch and
        one HBM round trip fewer than Normalize's spatial-major kernel + the transform; x needs no
        gradient)."""
        n = x.shape[-1]
        Q = self._take_spectral(n, x.device)
        return _SpectralConvFn.apply(x, Q, self.bias, n, False, groupsort, (mu, sd))

    def forward_hwcb(self, x: torch.Tensor) -> torch.Tensor:
        """The same map on spatial-major activations [n, n, C, B] (the conv stack's HBM layout):
        the 2-D rFFT over dims (0, 1) yields [n (n/2+1), C, B] = the per-frequency GEMM operand
        directly, the GEMM output is the inverse FFT's input, and the bias is added on the DC
        frequency (irfft2's 1/n^2 normalisation: + n^2 b), so no permute copies and no full-size
        bias pass."""
        if self.downsample:
            h, w, c, b = x.shape
            x = x.reshape(h // 2, 2, w // 2, 2, c, b).permute(0, 2, 4, 1, 3, 5).reshape(h // 2, w // 2, c * 4, b)
        cout, cin = self.weight.shape[:2]
        n, _, _, B = x.shape
        nf = n * (n // 2 + 1)
        xf = torch.fft.rfft2(x, dim=(0, 1)).reshape(nf, cin, B)
        Q = self._take_spectral(n, x.device)
        yf = Q @ xf
        if self.bias is not None:
            yf[0] += (float(n * n) * self.bias)[:, None]
        return torch.fft.irfft2(yf.reshape(n, n // 2 + 1, cout, B), s=(n, n), dim=(0, 1))
