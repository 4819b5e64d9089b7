"""The train_ode branch with torchdiffeq's adaptive dopri5 (cifar_train.yaml:30,32 train_ode_solver:
dopri5, train_ode_tol: 1e-3; pl_modules.py:490-500, models.py:235-241, use_adjoint False at
pl_modules.py:303) -- TEST INFRASTRUCTURE ONLY.

torchdiffeq 0.2.2 (env.yml:251) is absent from this image; its RKAdaptiveStepsizeODESolver is
restated here from its published algorithm (the same restatement as fiode_oracle.dopri5, whose
NFE / accept / reject sequence the device's eval solve reproduces):

  _select_initial_step(order 4):  d0 = rms(y0/s), d1 = rms(f0/s), s = atol + |y0| rtol,
      h0 = 1e-6 if d0 < 1e-5 or d1 < 1e-5 else 0.01 d0/d1;  f1 = f(y0 + h0 f0);
      d2 = rms((f1 - f0)/s)/h0;  h1 = max(1e-6, 1e-3 h0) if d1, d2 <= 1e-15 else (0.01/max(d1,d2))^(1/5);
      dt = min(100 h0, h1)  (then float64 time)
  _adaptive_step:  FSAL Dormand-Prince stages with dt cast to the state dtype, y1 = the 6th stage
      input, err = k (c_error dt), ratio = rms(err / (atol + rtol max(|y0|, |y1|))), accept iff
      ratio <= 1, interp coefficients from (y0, y1, y_mid = y0 + k (c_mid dt), f0, f1, dt);
  _optimal_step_size(order 5):  dt * (10 if ratio == 0 else min(10, max(0.9 ratio^-1/5, 1 if
      ratio < 1 else 0.2)))  in float64;
  output at t1: the dense interpolant of the last accepted step at x = (t1 - t0)/(t_next - t0).

Direct backprop (use_adjoint False) differentiates ALL of it: the stages, the error ratio of
accepted AND rejected attempts (they set the next step size), the step-size controller, the
initial-step selection and the interpolation point x (t_next = t0 + dt carries dt's gradient).

* ``dopri5_train``: the differentiable forward in torch (autograd = the reference's gradient).
* ``dopri5_adjoint``: the same gradient by a hand-written reverse sweep over a saved forward --
  the scheme the HIP backward (k_odp_bwd) implements -- using per-eval VJPs of the dynamics; the CPU
  suite checks it against autograd, so the device backward is pinned to autograd through it.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from oracle import fiode_oracle as O
from oracle import torch_ref as T

SAFETY, IFACTOR, DFACTOR = 0.9, 10.0, 0.2


def _rms(t):
    return t.abs().pow(2).mean().sqrt()


class Trace:
    """What the forward saw: per eval its input (a leaf when ``leaf_inputs``) and output, per
    attempt the controller's values, the initial-step scalars."""

    def __init__(self):
        self.Y: List[torch.Tensor] = []         # eval inputs
        self.K: List[torch.Tensor] = []         # eval outputs
        self.attempts: List[dict] = []
        self.init: dict = {}


def dopri5_train(x_feat, h0, W: Dict[str, torch.Tensor], masks=None, t0=0.0, t1=1.0, rtol=1e-3, atol=1e-3, *,
                 alpha_1=100.0, alpha_2=20.0, sigma_1=0.02, scale_nominal=True, p=0.5, acts=None, mus=None,
                 accepts=None, max_attempts=64, leaf_inputs=False, trace: Optional[Trace] = None):
    """y_hat = odeint(h_dot, h0, [t0, t1], method='dopri5', rtol, atol) in train mode, differentiable.
    masks: [E,2,B,M] keep masks of the e-th func() call; acts / mus: pinned QP active sets / exit mu
    per eval (torch_ref.eval_dot); accepts: pinned accept decisions per attempt.  leaf_inputs:
    every eval's input is detached into a leaf (its VJP alone, for dopri5_adjoint)."""
    dt_ = h0.dtype
    e = [0]

    def f(hh):
        i = e[0]
        e[0] += 1
        if leaf_inputs:
            hh = hh.detach().requires_grad_(True)
        m1 = masks[i, 0] if masks is not None else None
        m2 = masks[i, 1] if masks is not None else None
        k = T.eval_dot(hh, x_feat, W, alpha_1, alpha_2, sigma_1, scale_nominal, m1, m2, p,
                       act=None if acts is None else acts[i], mu=None if mus is None else mus[i])
        if trace is not None:
            trace.Y.append(hh)
            trace.K.append(k)
        return k

    beta = [[float(c) for c in row] for row in O.DOPRI5_BETA]
    cerr = [float(c) for c in O.DOPRI5_C_ERROR]
    cmid = [float(c) for c in O.DOPRI5_C_MID]
    rt = torch.tensor(rtol, dtype=dt_)
    at = torch.tensor(atol, dtype=dt_)
    y0 = h0
    f0 = f(y0)
    scale = at + y0.abs() * rt
    d0 = _rms(y0 / scale)
    d1 = _rms(f0 / scale)
    clamp0 = bool(d0 < 1e-5) or bool(d1 < 1e-5)
    hs = torch.tensor(1e-6, dtype=dt_) if clamp0 else 0.01 * d0 / d1
    y1i = y0 + hs * f0
    f1 = f(y1i)
    d2 = _rms((f1 - f0) / scale) / hs
    clamp1 = bool(d1 <= 1e-15) and bool(d2 <= 1e-15)
    if clamp1:
        h1 = torch.maximum(torch.tensor(1e-6, dtype=dt_), hs * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1.0 / 5.0)            # python max: d2 only if d2 > d1
    dt = torch.minimum(100 * hs, h1).to(torch.float64)
    if trace is not None:
        trace.init = dict(d0=d0, d1=d1, d2=d2, h0=hs, h1=h1, clamp0=clamp0, clamp1=clamp1, dt=dt)
    tcur = torch.tensor(t0, dtype=torch.float64)
    tmax = torch.tensor(t1, dtype=torch.float64)
    y, fcur = y0, f0
    tprev = tnext = tcur
    interp = None
    n = 0
    while bool(tmax > tnext):
        if n >= max_attempts:
            raise RuntimeError("dopri5_train: too many attempts")
        dts = dt.to(dt_)
        ta = tcur + dt
        k = [fcur]
        for i in range(6):
            acc = k[0] * (beta[i][0] * dts)
            for j in range(1, i + 1):
                acc = acc + k[j] * (beta[i][j] * dts)
            yi = y + acc
            k.append(f(yi))
        ynew = yi
        err = k[0] * (cerr[0] * dts)
        for j in range(1, 7):
            err = err + k[j] * (cerr[j] * dts)
        etol = at + rt * torch.maximum(y.abs(), ynew.abs())
        ratio = _rms(err / etol)
        accept = bool(ratio <= 1) if accepts is None else bool(accepts[n])
        rec = dict(t=tcur, dt=dt, ratio=ratio, accept=accept)
        if accept:
            ym = k[0] * (cmid[0] * dts)
            for j in range(1, 7):
                ym = ym + k[j] * (cmid[j] * dts)
            ymid = y + ym
            fa, fb = k[0], k[6]
            a = 2 * dts * (fb - fa) - 8 * (ynew + y) + 16 * ymid
            b = dts * (5 * fa - 3 * fb) + 18 * y + 14 * ynew - 32 * ymid
            c = dts * (fb - 4 * fa) - 11 * y - 5 * ynew + 16 * ymid
            d = dts * fa
            interp = [y, d, c, b, a]
            tprev, tnext = tcur, ta
            y, fcur, tcur = ynew, fb, ta
        n += 1
        r64 = ratio.to(torch.float64)
        if bool(r64 == 0):
            dt = dt * IFACTOR
            rec["fmode"] = "zero"
        else:
            df = 1.0 if bool(r64 < 1) else DFACTOR
            mid = SAFETY / r64 ** (1.0 / 5.0)
            mf = float(mid.detach())
            rec["fmode"] = "mid" if (df < mf < IFACTOR) else ("hi" if mf >= IFACTOR else "lo")
            dt = dt * torch.minimum(torch.tensor(IFACTOR, dtype=torch.float64),
                                    torch.maximum(mid, torch.tensor(df, dtype=torch.float64)))
        if trace is not None:
            trace.attempts.append(rec)
    x = ((tmax - tprev) / (tnext - tprev)).to(dt_)
    total = interp[0] + x * interp[1]
    xp = x
    for coef in interp[2:]:
        xp = xp * x
        total = total + xp * coef
    return total, dict(nfe=e[0], n_attempts=n, accepts=[r["accept"] for r in (trace.attempts if trace else [])])


def dopri5_adjoint(tr: Trace, g_out: torch.Tensor, params: Dict[str, torch.Tensor], t0=0.0, t1=1.0, rtol=1e-3,
                   atol=1e-3):
    """The reverse sweep of k_odp_bwd over a saved forward (``dopri5_train(..., leaf_inputs=True,
    trace=tr)``): returns the parameter gradients of <g_out, y_hat>.  Every eval's VJP comes from
    its own graph (torch.autograd.grad of K[e] w.r.t. its leaf input and the parameters); the RK
    structure, the error ratio, the step-size controller, the initial-step selection and the
    interpolation point are differentiated by hand, in the order the kernel runs them:
      attempts in reverse; per attempt: scalar adjoints (dt_{n+1} -> ratio_n, dt_n), the row
      adjoints of y_{n+1} / f_{n+1} (accepted) or their pass-through (rejected), the error ratio's
      row terms, stages 6..1 (VJP, then the stage-input sum), one batch reduction of the dt
      partials; then the initial step (two more reductions)."""
    beta = [[float(c) for c in row] for row in O.DOPRI5_BETA]
    cerr = [float(c) for c in O.DOPRI5_C_ERROR]
    cmid = [float(c) for c in O.DOPRI5_C_MID]
    grads = {k: torch.zeros_like(v) for k, v in params.items()}
    keys = list(params)
    Y, K = tr.Y, tr.K
    A = len(tr.attempts)
    N = g_out.numel()

    def vjp(e, gk):
        outs = torch.autograd.grad(K[e], [Y[e]] + [params[k] for k in keys], gk, retain_graph=True,
                                   allow_unused=True)
        for k, g in zip(keys, outs[1:]):
            if g is not None:
                grads[k] += g
        return outs[0]

    at, rt = atol, rtol
    # the forward state per attempt: y_n (the attempt's base), the eval index of its k_0
    ys, fidx = [], []
    y = Y[0].detach()
    fi = 0
    e = 2
    for n, rec in enumerate(tr.attempts):
        ys.append(y)
        fidx.append(fi)
        if rec["accept"]:
            y = Y[e + 5].detach()            # y_new = the 6th stage input
            fi = e + 5                       # FSAL: k_6 of this attempt (eval e + 5)
        e += 6
    L = A - 1
    gy = torch.zeros_like(g_out)             # adjoint of the running state y_{n+1}
    gf = torch.zeros_like(g_out)             # adjoint of f_{n+1}
    g_dt_next = 0.0                          # adjoint of dt_{n+1}
    g_t_next = 0.0                           # adjoint of t_{n+1}
    for n in range(A - 1, -1, -1):
        rec = tr.attempts[n]
        e0 = 2 + 6 * n                       # evals of k_1..k_6: e0 .. e0 + 5
        dt = float(rec["dt"])
        dts = float(rec["dt"].to(g_out.dtype))
        ratio = float(rec["ratio"])
        # controller: dt_{n+1} = dt_n factor(ratio_n)
        if rec["fmode"] == "zero":
            fac, dfac = IFACTOR, 0.0
        else:
            df = 1.0 if ratio < 1 else DFACTOR
            mid = SAFETY / ratio ** 0.2
            fac = min(IFACTOR, max(mid, df))
            dfac = -0.2 * mid / ratio if rec["fmode"] == "mid" else 0.0
        g_ratio = g_dt_next * dt * dfac
        g_dt = g_dt_next * fac
        kk = [K[fidx[n]].detach()] + [K[e0 + i].detach() for i in range(6)]
        yn = ys[n]
        ynew = Y[e0 + 5].detach()
        gk = [torch.zeros_like(g_out) for _ in range(7)]
        g_yn = torch.zeros_like(g_out)
        g_ynew = torch.zeros_like(g_out)
        g_dts = 0.0
        g_x = 0.0
        if rec["accept"]:
            g_ynew += gy
            gk[6] += gf
        else:
            g_yn += gy
            gk[0] += gf
        if n == L:                           # the output: interpolant at x
            tprev = float(rec["t"])
            x64 = (t1 - tprev) / ((tprev + dt) - tprev)
            x = float(torch.tensor(x64, dtype=g_out.dtype))
            ym = yn + sum(kk[j] * (cmid[j] * dts) for j in range(7))
            fa, fb = kk[0], kk[6]
            a = 2 * dts * (fb - fa) - 8 * (ynew + yn) + 16 * ym
            b = dts * (5 * fa - 3 * fb) + 18 * yn + 14 * ynew - 32 * ym
            c = dts * (fb - 4 * fa) - 11 * yn - 5 * ynew + 16 * ym
            d = dts * fa
            ga, gb, gc, gd, ge = g_out * x ** 4, g_out * x ** 3, g_out * x ** 2, g_out * x, g_out
            g_x = float((g_out * (d + 2 * x * c + 3 * x ** 2 * b + 4 * x ** 3 * a)).sum())
            g_ym = 16 * ga - 32 * gb + 16 * gc
            g_yn += ge - 8 * ga + 18 * gb - 11 * gc
            g_ynew += -8 * ga + 14 * gb - 5 * gc
            gfa = -2 * dts * ga + 5 * dts * gb - 4 * dts * gc + dts * gd
            gfb = 2 * dts * ga - 3 * dts * gb + dts * gc
            g_dts += float((ga * 2 * (fb - fa) + gb * (5 * fa - 3 * fb) + gc * (fb - 4 * fa) + gd * fa).sum())
            g_yn += g_ym
            for j in range(7):
                gk[j] += g_ym * (cmid[j] * dts)
                g_dts += float((g_ym * kk[j] * cmid[j]).sum())
            gk[0] += gfa
            gk[6] += gfb
        # error ratio: ratio = rms(q), q = err / etol, etol = atol + rtol max(|y_n|, |y_new|)
        if g_ratio != 0.0:
            err = sum(kk[j] * (cerr[j] * dts) for j in range(7))
            etol = at + rt * torch.maximum(yn.abs(), ynew.abs())
            q = err / etol
            gq = g_ratio * q / (N * ratio)
            g_err = gq / etol
            g_etol = -gq * q / etol
            pick_n = yn.abs() >= ynew.abs()
            g_yn += torch.where(pick_n, g_etol * rt * torch.sign(yn), torch.zeros_like(yn))
            g_ynew += torch.where(pick_n, torch.zeros_like(yn), g_etol * rt * torch.sign(ynew))
            for j in range(7):
                gk[j] += g_err * (cerr[j] * dts)
                g_dts += float((g_err * kk[j] * cerr[j]).sum())
        # stages in reverse: k_{i+1} = f(Y_i), Y_i = y_n + sum_{j<=i} k_j beta_ij dt; y_new = Y_5
        gY = [torch.zeros_like(g_out) for _ in range(6)]
        gY[5] += g_ynew
        for i in range(5, -1, -1):
            gY[i] = gY[i] + vjp(e0 + i, gk[i + 1])
            g_yn += gY[i]
            for j in range(i + 1):
                gk[j] += gY[i] * (beta[i][j] * dts)
                g_dts += float((gY[i] * kk[j] * beta[i][j]).sum())
        # one batch reduction: sum of the dt partials (and g_x)
        g_dt += g_dts
        if n == L:
            span = dt
            g_dt += -g_x * x64 / span            # x = (t1 - t_L)/(t_L + dt - t_L)
            g_t = -g_x / span
        else:
            g_t = g_t_next
        if rec["accept"] and n != L:
            g_dt += g_t_next                     # t_{n+1} = t_n + dt_n
        g_t_next = g_t
        g_dt_next = g_dt
        gy = g_yn
        gf = gk[0]
    # ---- the initial step: dt_0 = min(100 h0, h1) ---------------------------------------------
    ini = tr.init
    s = at + Y[0].detach().abs() * rt
    f0, f1 = K[0].detach(), K[1].detach()
    h0, h1 = float(ini["h0"]), float(ini["h1"])
    d1, d2 = float(ini["d1"]), float(ini["d2"])
    d0 = float(ini["d0"])
    g_h0 = g_dt_next * 100 if 100 * h0 <= h1 else 0.0
    g_h1 = g_dt_next if h1 < 100 * h0 else 0.0
    g_d1 = g_d2 = 0.0
    if ini["clamp1"]:
        if h0 * 1e-3 > 1e-6:
            g_h0 += 1e-3 * g_h1
    else:
        m = d2 if d2 > d1 else d1
        g_m = g_h1 * (-0.2) * h1 / m
        if d2 > d1:
            g_d2 += g_m
        else:
            g_d1 += g_m
    # d2 = rms((f1 - f0)/s) / h0
    r2 = d2 * h0
    g_r2 = g_d2 / h0
    g_h0 += -g_d2 * d2 / h0
    w = (f1 - f0) / s
    g_w = g_r2 * w / (N * r2) if r2 > 0 else torch.zeros_like(w)
    g_f1 = g_w / s
    g_f0 = gf - g_w / s                       # gf: the adjoint of f_0 = k_0 of attempt 0
    g_y1i = vjp(1, g_f1)
    g_f0 = g_f0 + h0 * g_y1i
    g_h0 += float((g_y1i * f0).sum())         # batch reduction
    if not ini["clamp0"]:
        g_d1 += -g_h0 * h0 / d1               # h0 = 0.01 d0 / d1
    q1 = f0 / s
    g_f0 = g_f0 + (g_d1 * q1 / (N * d1)) / s
    vjp(0, g_f0)
    return grads
