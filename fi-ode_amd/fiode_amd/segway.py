"""BASELINE configs[0]: the Segway safe-control plumbing check, on the CPU.

The reference trains a 3-state Segway controller (control/train_segway.py:23-209) and plots its
closed-loop trajectories with ``system.simulate(x_0, nn_controller, ts)`` over
``ts = linspace(0, 50, 10000)`` for 5 initial states (control/certify_segway.py:104-109).  The
Segway model, ``NNController(system, 3, 1, 32)``, ``LinearController`` and ``simulate`` live in the
``libs/core`` submodule, which is EMPTY in the reference tree (.gitmodules:1-12), so this module
restates the interfaces the reference calls with a reduced 3-state model of our own:

    x = (phi, v, phi_dot),  x' = f(x) + g u,
    f(x) = (phi_dot, a_v sin(phi) - d_v v, a_p sin(phi) - d_p v),  g = (0, b_v, -b_p),

linearised for the LQR start of the controller exactly as train_segway.py:31-43 does
(system.jacobian at the goal, scipy solve_continuous_are, K = R^-1 G^T P).  ``simulate`` integrates
the closed loop with ``fiode_amd.odeint.odeint(..., method='rk4')`` -- torchdiffeq's fixed grid on
``ts`` itself -- on whatever device the state lives (configs[0] is CPU-only plumbing).  Parity of
the model with the absent ``libs/core`` is UNPINNED; the integrator is pinned against the oracle's
``rk4_on_grid`` (tests/test_segway.py).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
import torch.nn as nn

from .odeint import odeint


class Segway(nn.Module):
    """Reduced 3-state Segway (restated; see the module docstring)."""

    n, m = 3, 1

    def __init__(self, a_v: float = 4.0, d_v: float = 1.5, a_p: float = 12.0, d_p: float = 0.4,
                 b_v: float = 1.2, b_p: float = 1.8):
        super().__init__()
        self.a_v, self.d_v, self.a_p, self.d_p, self.b_v, self.b_p = a_v, d_v, a_p, d_p, b_v, b_p

    def drift(self, x: torch.Tensor, t=0.0) -> torch.Tensor:
        phi, v, dphi = x.unbind(-1)
        s = torch.sin(phi)
        return torch.stack([dphi, self.a_v * s - self.d_v * v, self.a_p * s - self.d_p * v], -1)

    def act(self, x: torch.Tensor, t=0.0) -> torch.Tensor:
        g = torch.tensor([0.0, self.b_v, -self.b_p], dtype=x.dtype, device=x.device)
        return g.expand(*x.shape[:-1], 3)[..., None]                   # [.., 3, 1]

    def forward(self, x: torch.Tensor, u: torch.Tensor, t=0.0) -> torch.Tensor:
        return self.drift(x, t) + (self.act(x, t) @ u[..., None])[..., 0]

    def jacobian(self, x: torch.Tensor, u: torch.Tensor, t=0.0) -> Tuple[torch.Tensor, torch.Tensor]:
        """(d f / d x, d f / d u) at (x, u): [B, 3, 3], [B, 3, 1] (train_segway.py:35)."""
        F = torch.stack([torch.autograd.functional.jacobian(lambda z: self(z[None], u[i:i + 1], t)[0], x[i])
                         for i in range(x.shape[0])])
        G = torch.stack([torch.autograd.functional.jacobian(lambda w: self(x[i:i + 1], w[None], t)[0], u[i])
                         for i in range(x.shape[0])])
        return F, G

    def closed_loop(self, controller):
        def f(t, x):
            return self(x, controller(x, t), t)
        return f

    def simulate(self, x0: torch.Tensor, controller, ts) -> Tuple[torch.Tensor, torch.Tensor]:
        """Closed-loop states [B, T, 3] and inputs [B, T, 1] at ts (certify_segway.py:108-109):
        odeint with method='rk4' on the grid ts (no step_size: torchdiffeq's grid = ts)."""
        ts = torch.as_tensor(np.asarray(ts), dtype=x0.dtype, device=x0.device)
        xs = odeint(self.closed_loop(controller), x0, ts, method="rk4")       # [T, B, 3]
        xs = xs.transpose(0, 1).contiguous()
        with torch.no_grad():
            us = controller(xs.reshape(-1, 3), 0.0).reshape(xs.shape[0], xs.shape[1], 1)
        return xs, us


class LinearController(nn.Module):
    """u = -K x (train_segway.py:43)."""

    def __init__(self, system, K: torch.Tensor):
        super().__init__()
        self.system = system
        self.register_buffer("K", torch.as_tensor(K, dtype=torch.float32))

    def forward(self, x, t=0.0):
        return -x @ self.K.T


class NNController(nn.Module):
    """NNController(system, n_in, n_out, hidden) (train_segway.py:49): an MLP state feedback,
    u = W3 tanh(W2 tanh(W1 x + b1) + b2) + b3, plus an optional fixed linear term -K x (the LQR
    start that train_segway.py:52-68 fits the MLP to)."""

    def __init__(self, system, n_in: int = 3, n_out: int = 1, hidden: int = 32, K=None):
        super().__init__()
        self.system = system
        self.net = nn.Sequential(nn.Linear(n_in, hidden), nn.Tanh(), nn.Linear(hidden, hidden), nn.Tanh(),
                                 nn.Linear(hidden, n_out))
        self.register_buffer("K", torch.zeros(n_out, n_in) if K is None else torch.as_tensor(K, dtype=torch.float32))

    def forward(self, x, t=0.0):
        return self.net(x) - x @ self.K.T


def lqr_gain(system: Segway, Q=None, R=None) -> torch.Tensor:
    """K = R^-1 G^T P with P from the continuous ARE at the goal (train_segway.py:31-43)."""
    from scipy.linalg import solve_continuous_are
    Q = 10 * np.eye(3) if Q is None else np.asarray(Q)
    R = np.eye(1) if R is None else np.asarray(R)
    goal = torch.zeros(1, 3)
    F, G = system.jacobian(goal, torch.zeros(1, 1), 0.0)
    P = solve_continuous_are(a=F[0].detach().numpy(), b=G[0].detach().numpy(), q=Q, r=R)
    return torch.tensor(np.linalg.inv(R) @ G[0].detach().numpy().T @ P, dtype=torch.float32)
