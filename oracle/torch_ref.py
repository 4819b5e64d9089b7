"""Op-for-op torch-CPU restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

Used (a) to pin ``oracle/fiode_oracle.py``'s closed-form backward against the reference's own
autograd semantics (``torch.autograd.functional.jvp(create_graph=True)`` through
DecisionBoundary, the QP ``autograd.Function`` with dense (N,C,C) Jacobian masks, dropout,
ReLU, F.linear), and (b) as the CPU baseline that ``bench.py`` times (``cpu_baseline.kind`` =
"port"): it runs the reference algorithm the way the reference runs it, one eager torch op
at a time, on the host cores.

Written from the reference source text (never imported):
  classification.py:96-126, barrier_projection.py:217-313, lya_cands.py:79-94,
  pl_modules.py:390-484, sampler.py:34-38,113-128,195-216.
The Cayley effective weights are passed in (their body lives in the absent ortho_conv lib).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch.autograd import Function
from torch.autograd.functional import jvp


class _NoUpperProjection(Function):
    """barrier_projection.py:217-313 restated: batch-global bisection forward (with the
    per-iteration ``max|eps| < tol`` host check), dense-mask Jacobian backward."""

    max_iter = 30
    tol = 1e-4

    @staticmethod
    def forward(ctx, lower, nominal):
        with torch.no_grad():
            n = nominal.shape[0]
            mu = torch.zeros((n, 1), dtype=nominal.dtype)
            hi = torch.ones_like(mu) * (nominal - lower).max(dim=-1).values[:, None]
            lo = torch.ones_like(mu) * nominal.min(dim=-1).values[:, None]
            v = torch.zeros_like(nominal)
            for _ in range(_NoUpperProjection.max_iter):
                mu = (hi - lo) / 2 + lo
                v.copy_(nominal)
                v -= mu
                v.clamp_(lower)
                eps = v.sum(dim=-1)[:, None]
                if eps.abs().max() < _NoUpperProjection.tol:
                    break
                lo = torch.where(eps > 0, mu, lo)
                hi = torch.where(eps < 0, mu, hi)
        ctx.save_for_backward(v, mu, lower, nominal)
        return v

    @staticmethod
    def backward(ctx, g):
        v, mu, lower, nominal = ctx.saved_tensors
        n, c = v.shape
        act = (v - nominal + mu) > 0
        na = ~act
        rec_na = (1 / na.sum(dim=-1).to(g.dtype))[:, None, None].expand(-1, c, c)
        eye = torch.eye(c, dtype=torch.bool)[None]
        jn = torch.zeros((n, c, c), dtype=g.dtype)
        m = na[:, None, :] & na[:, :, None]
        jn[m] = -rec_na[m]
        jn[eye & na[:, :, None]] += 1
        jl = torch.zeros((n, c, c), dtype=g.dtype)
        m2 = act[:, None, :] & na[:, :, None]
        jl[m2] = -rec_na[m2]
        jl[eye & act[:, :, None]] += 1
        return (g[:, None, :] @ jl)[:, 0, :], (g[:, None, :] @ jn)[:, 0, :]


class _PinnedActiveSet(Function):
    """The same projection whose backward takes its active set from another implementation's
    (v, mu, nominal) -- the QP active-set test ``(v - nominal) + mu > 0`` is float32 rounding
    noise for inactive coordinates (see fiode_oracle.eval_dot), so chained checks pin it."""

    @staticmethod
    def forward(ctx, lower, nominal, act, mu=None):
        if mu is None:
            v = _NoUpperProjection.forward(ctx, lower, nominal)
        else:       # the exit iteration's mu pinned too: v = max(nominal - mu, lower) (:242-244)
            v = torch.maximum(nominal - mu.to(nominal.dtype)[:, None], lower)
        ctx.act = act
        return v

    @staticmethod
    def backward(ctx, g):
        act = ctx.act
        na = ~act
        cnt = na.sum(dim=-1, keepdim=True).to(g.dtype)
        corr = torch.where(cnt > 0, (g * na).sum(dim=-1, keepdim=True) / cnt.clamp(min=1), torch.zeros_like(cnt))
        d = g - corr
        return torch.where(act, d, torch.zeros_like(d)), torch.where(act, torch.zeros_like(d), d), None, None


def eval_dot(h, x_rows, W: Dict[str, torch.Tensor], alpha_1, alpha_2, sigma_1, scale_nominal,
             mask1=None, mask2=None, p=0.5, stash=None, act=None, mu=None):
    """classification.py:96-115 (eval_dot) with dropout masks injected.  ``stash`` (a dict)
    receives the QP inputs (lower, nominal) so a checker can pin the QP's active-set test."""
    z = F.linear(h, W["Q1"], W["b1"]) + F.linear(x_rows, W["Qx"], W["bx"])
    if mask1 is not None:
        z = z * (mask1.to(z.dtype) * (1.0 / (1.0 - p)))
    a = torch.relu(z)
    z = F.linear(a, W["Q2"], W["b2"])
    if mask2 is not None:
        z = z * (mask2.to(z.dtype) * (1.0 / (1.0 - p)))
    a = torch.relu(z)
    ft = F.linear(a, W["Q3"], W["b3"])
    lower = -alpha_1 * (torch.exp(sigma_1 * h) - 1)
    upper = alpha_2 * (1 - h)
    if scale_nominal:
        ft = (upper - lower) * torch.sigmoid(ft) + lower
    if stash is not None:
        stash["lower"] = lower.detach().clone()
        stash["nominal"] = ft.detach().clone()
    if act is not None:
        return _PinnedActiveSet.apply(lower, ft, act, mu)
    return _NoUpperProjection.apply(lower, ft)


def decision_boundary(prob, y):
    """lya_cands.py:79-94 (on_simplex=True, log_mode=False)."""
    prob_y = torch.gather(prob, dim=1, index=y[:, None])[:, 0]
    wrong = torch.masked_select(prob, ~F.one_hot(y, prob.shape[1]).bool())
    wrong = wrong.unflatten(0, (prob.shape[0], prob.shape[1] - 1))
    return 1 + wrong.max(dim=-1).values - prob_y


def lyapunov_loss(h, x_feat, y, S, W, *, alpha_1=100.0, alpha_2=20.0, sigma_1=0.02,
                  scale_nominal=True, kappa=2.0, p=0.5, mask1=None, mask2=None,
                  lmask1=None, lmask2=None, stash=None):
    """pl_modules.py:394-484 for order=1, act='relu', DecisionBoundary, no lips/barrier terms.
    Returns (loss, eff, mean_active)."""
    x_in = x_feat[:, None].expand(-1, S, -1).flatten(0, 1)
    y_in = y[:, None].expand(-1, S).flatten(0, 1)
    tangent = eval_dot(h, x_in, W, alpha_1, alpha_2, sigma_1, scale_nominal, mask1, mask2, p, stash)
    v, vd = jvp(func=lambda hh: decision_boundary(hh, y_in), inputs=(h,), v=tangent, create_graph=True)
    viol = torch.relu(vd + kappa * v.detach())
    eff = (viol > 0).sum()
    loss = viol.mean()
    with torch.no_grad():
        f = eval_dot(h, x_in, W, alpha_1, alpha_2, sigma_1, scale_nominal, lmask1, lmask2, p)
        lower = -alpha_1 * h
        upper = alpha_2 * (1 - h)
        act = ((f - lower).abs() <= 1e-6) | ((f - upper).abs() <= 1e-6)
        mean_active = act.float().mean()
    return loss, eff, mean_active


def step_with_grads(h, x_feat, y, S, W: Dict[str, torch.Tensor], **kw):
    """Forward + ``loss.backward()``; returns (loss, eff, mean_active, grads) with grads w.r.t.
    the effective weights/biases and the static features."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in W.items()}
    xf = x_feat.detach().clone().requires_grad_(True)
    loss, eff, ma = lyapunov_loss(h, xf, y, S, leaves, **kw)
    loss.backward()
    grads = {k: v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v) for k, v in leaves.items()}
    grads["x_feat"] = xf.grad.detach().clone()
    return float(loss.detach()), int(eff), float(ma), grads


def uniform_simplex(draws):
    """sampler.py:34-38 with the Exp(1) draws given."""
    return F.normalize(draws, p=1.0, dim=1)


def correct_cone(draws, y):
    """sampler.py:113-128 with the Exp(1) draws given ([B,S2,C])."""
    B, S2, C = draws.shape
    h = F.normalize(draws, dim=-1, p=1)
    mo = h.max(dim=-1)
    oh = F.one_hot(y, num_classes=C).bool()
    lab = h[oh[:, None, :].expand(-1, S2, -1)]
    h[oh[:, None, :].expand(-1, S2, -1)] = mo.values.flatten()
    h.scatter_(2, mo.indices[:, :, None], lab.unflatten(0, mo.indices.shape)[:, :, None])
    return h


def rk4_grid32(t0: float, t1: float, step_size: float):
    """FixedGridODESolver's float32 grid: niters = ceil((t1-t0)/h + 1), t_k = k h + t0, last = t1."""
    import math
    t0f, t1f, hf = torch.tensor(t0, dtype=torch.float32), torch.tensor(t1, dtype=torch.float32), \
        torch.tensor(step_size, dtype=torch.float32)
    n = int(math.ceil(float((t1f - t0f) / hf + 1)))
    g = torch.arange(n, dtype=torch.float32) * hf + t0f
    g[-1] = t1f
    return g


def ode_train_loss(x_feat, h0, y, W: Dict[str, torch.Tensor], masks, t0=0.0, t1=1.0, step_size=0.1, *,
                   alpha_1=100.0, alpha_2=20.0, sigma_1=0.02, scale_nominal=True, p=0.5, acts=None, mus=None):
    """pl_modules.py:490-497: y_hat = odeint(h_dot, h0, [t0, t1], method='rk4', step_size) in train
    mode (torchdiffeq 0.2.2 rk4_alt_step_func op order), loss_ode = nll_loss(log(y_hat), y).
    masks: [E,2,B,M] uint8 keep masks per func() call; acts: optional per-eval pinned QP active
    sets [E][B,C] bool; mus: optional per-eval pinned exit mu [E][B] (with acts: the linearisation
    points of another implementation's forward, so a float64 run checks its float32 backward).
    Returns (loss_ode, y_hat)."""
    grid = rk4_grid32(t0, t1, step_size)
    third = 1.0 / 3.0
    e = [0]

    def f(hh):
        i = e[0]
        e[0] += 1
        m1 = masks[i, 0] if masks is not None else None
        m2 = masks[i, 1] if masks is not None else None
        return eval_dot(hh, x_feat, W, alpha_1, alpha_2, sigma_1, scale_nominal, m1, m2, p,
                        act=None if acts is None else acts[i], mu=None if mus is None else mus[i])
    yy = h0
    for a, b in zip(grid[:-1], grid[1:]):
        dt = b - a
        k1 = f(yy)
        k2 = f(yy + dt * k1 * third)
        k3 = f(yy + dt * (k2 - k1 * third))
        k4 = f(yy + dt * (k1 - k2 + k3))
        yy = yy + (k1 + 3 * (k2 + k3) + k4) * dt * 0.125
    return F.nll_loss(torch.log(yy), y), yy
