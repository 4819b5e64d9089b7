"""torchdiffeq-compatible ``odeint`` (the call at models.py:235-241).

``odeint(func, y0, t, rtol, atol, method, options)`` with torchdiffeq 0.2.2's signature and
semantics.  When ``func`` is the h_dot of an IVP whose dynamics is the HIP-backed
OrthoClassDynProjectSimplexLips, the whole solve runs as ONE persistent gfx950 kernel
(fiode_odeint: RK4 3/8-rule fixed grid or dopri5 with the batch-global RMS error norm).  Any other
right-hand side (e.g. the 3-state Segway plumbing check of BASELINE config 1) runs the same two
algorithms as plain torch ops on whatever device its tensors live on.

make_solver_params (pl_modules.py:24-35) is reproduced: adaptive solvers take rtol=atol=tol;
fixed-grid solvers take options.step_size = tol.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

ADAPTIVE_SOLVERS = ["dopri8", "dopri5", "bosh3", "fehlberg2", "adaptive_heun", "scipy_solver"]
FIXED_SOVLERS = ["euler", "midpoint", "rk4", "explicit_adams", "implicit_adams", "fixed_adams"]


def make_solver_params(solver_name, ode_tol):
    """pl_modules.py:24-35."""
    if solver_name in ADAPTIVE_SOLVERS:
        return dict(method=solver_name, rtol=ode_tol, atol=ode_tol)
    if solver_name in FIXED_SOVLERS:
        return dict(method=solver_name, options=dict(step_size=ode_tol))
    raise RuntimeError("[ERROR] Invalid Solver Name")


def _native_target(func):
    """The HIP-backed dynamics behind ``func``: an IVP's ``h_dot`` (models.py:200-201) or the
    dynamics' own ``ode_forward`` (classification.py:128-132), else None."""
    from .dynamics import OrthoClassDynProjectSimplexLips
    owner = getattr(func, "__self__", None)
    name = getattr(func, "__name__", "")
    if isinstance(owner, OrthoClassDynProjectSimplexLips) and name == "ode_forward":
        return owner
    dyn = getattr(owner, "dyn_fun", None)
    if isinstance(dyn, OrthoClassDynProjectSimplexLips) and name == "h_dot":
        return dyn
    return None


def odeint(func, y0, t, rtol=1e-7, atol=1e-9, method=None, options=None, **unused):
    method = method or "dopri5"
    options = dict(options or {})
    is_tuple = isinstance(y0, tuple)
    y = y0[0] if is_tuple else y0
    if is_tuple and len(y0) != 1:
        raise NotImplementedError("tupled states with more than one tensor")
    dyn = _native_target(func)
    if dyn is not None:
        sol = _odeint_native(dyn, y, t, rtol, atol, method, options)
    else:
        sol = _odeint_torch(lambda tt, yy: func(tt, (yy,) if is_tuple else yy), y, t, rtol, atol, method, options,
                            tuple_out=is_tuple)
    return (sol,) if is_tuple else sol


def _odeint_native(dyn, h0, t, rtol, atol, method, options):
    from . import ops
    if dyn.static_state is None:
        raise RuntimeError("[ERROR] You forgot to set static state before calling forward.")
    if dyn.training and dyn.dropout.p > 0:
        raise NotImplementedError("odeint through the training-mode (dropout) dynamics is not fused; "
                                  "validation/inference solves run in eval mode")
    times = t.detach().to(device=h0.device, dtype=torch.float64)
    with torch.no_grad():
        w = {k: v.detach().float().contiguous() for k, v in dyn.effective_weights().items()}
        sol, stats, dstats = ops.odeint_dyn(dyn.static_state.detach().float().contiguous(),
                                            h0.detach().float().contiguous(), times, w, dyn.dyn_cfg(),
                                            method=method, rtol=float(rtol), atol=float(atol),
                                            step_size=options.get("step_size"),
                                            max_steps=int(options.get("max_num_steps", 100000)))
    dyn.last_solve_stats = (stats, dstats)
    status = int(stats[3])        # one host read per solve (torchdiffeq raises here too)
    if status == 2:
        raise RuntimeError(f"max_num_steps exceeded ({int(stats[5])} steps)")
    if status == 3:
        raise AssertionError(f"underflow in dt {float(dstats[0])}")
    if status:
        raise RuntimeError(f"fiode_odeint: cross-workgroup exchange timed out (status {status}); results invalid")
    return sol


# ---- generic torch steppers (same algorithms, any func / device) --------------------------------

def _rk4_grid(t0: torch.Tensor, t1: torch.Tensor, h: float, dtype):
    niters = int(torch.ceil((t1 - t0) / h + 1).item())
    g = torch.arange(0, niters, dtype=dtype, device=t0.device) * h + t0
    g[-1] = t1
    return g


def _odeint_torch(f, y0, t, rtol, atol, method, options, tuple_out=False):
    def F(tt, yy):
        out = f(tt, yy)
        return out[0] if isinstance(out, tuple) else out

    if method == "rk4":
        h = options.get("step_size")
        # torchdiffeq 0.2.2 FixedGridODESolver: options.step_size builds the grid
        # (_grid_constructor_from_step_size); without it the grid is t itself
        grid = t if h is None else _rk4_grid(t[0], t[-1], h, t.dtype)
        sol = [y0]
        j = 1
        y = y0
        third = 1.0 / 3.0
        for a, b in zip(grid[:-1], grid[1:]):
            dt = b - a
            k1 = F(a, y)
            k2 = F(a + dt * third, y + dt * k1 * third)
            k3 = F(a + dt * (2.0 / 3.0), y + dt * (k2 - k1 * third))
            k4 = F(b, y + dt * (k1 - k2 + k3))
            y1 = y + (k1 + 3 * (k2 + k3) + k4) * dt * 0.125
            while j < len(t) and b >= t[j]:
                if t[j] == a:
                    sol.append(y)
                elif t[j] == b:
                    sol.append(y1)
                else:
                    sol.append(y + (t[j] - a) / (b - a) * (y1 - y))
                j += 1
            y = y1
        return torch.stack(sol)
    if method == "dopri5":
        return _dopri5_torch(F, y0, t, rtol, atol, options)
    raise NotImplementedError(f"method {method!r}")


_BETA = [[1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9],
         [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
         [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
         [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]]
_CERR = [35 / 384 - 1951 / 21600, 0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
         -2187 / 6784 - -12231 / 42400, 11 / 84 - 649 / 6300, -1.0 / 60.0]
_CMID = [6025192743 / 30085553152 / 2, 0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
         187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2]


def _rms(x):
    return x.abs().pow(2).mean().sqrt()


def _dopri5_torch(F, y0, t, rtol, atol, options):
    safety, ifactor, dfactor = 0.9, 10.0, 0.2
    t = t.to(torch.float64)
    y = y0
    f0 = F(t[0], y)
    scale = atol + y.abs() * rtol
    d0, d1 = _rms(y / scale), _rms(f0 / scale)
    h0 = torch.tensor(1e-6, dtype=y.dtype) if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    f1 = F(t[0] + h0, y + h0 * f0)
    d2 = _rms((f1 - f0) / scale) / h0
    h1 = torch.max(torch.tensor(1e-6, dtype=y.dtype), h0 * 1e-3) if (d1 <= 1e-15 and d2 <= 1e-15) \
        else (0.01 / max(d1, d2)) ** (1.0 / 5.0)
    dt = float(torch.min(100 * h0, h1))
    tcur, tprev, tnext = float(t[0]), float(t[0]), float(t[0])
    fcur, interp = f0, None
    sol = [y0]
    for tout in t[1:].tolist():
        while tout > tnext:
            ta = tcur + dt
            k = [fcur]
            for i in range(6):
                acc = sum(k[j] * (_BETA[i][j] * dt) for j in range(i + 1))
                k.append(F(ta if i >= 4 else tcur + [1 / 5, 3 / 10, 4 / 5, 8 / 9][i] * dt, y + acc))
            ynew = y + sum(k[j] * (_BETA[5][j] * dt) for j in range(6))
            err = sum(k[j] * (_CERR[j] * dt) for j in range(7))
            ratio = float(_rms(err / (atol + rtol * torch.maximum(y.abs(), ynew.abs()))))
            if ratio <= 1:
                ym = y + sum(k[j] * (_CMID[j] * dt) for j in range(7))
                fa, fb = k[0], k[6]
                interp = [y, dt * fa, dt * (fb - 4 * fa) - 11 * y - 5 * ynew + 16 * ym,
                          dt * (5 * fa - 3 * fb) + 18 * y + 14 * ynew - 32 * ym,
                          2 * dt * (fb - fa) - 8 * (ynew + y) + 16 * ym]
                tprev, tnext = tcur, ta
                y, fcur, tcur = ynew, k[6], ta
            dt = dt * ifactor if ratio == 0 else dt * min(ifactor, max(safety / ratio ** 0.2, 1.0 if ratio < 1 else dfactor))
        x = (tout - tprev) / (tnext - tprev)
        total = interp[0] + x * interp[1]
        xp = x
        for c in interp[2:]:
            xp = xp * x
            total = total + xp * c
        sol.append(total)
    return torch.stack(sol)
