"""BASELINE configs[0] (CPU): the Segway closed loop simulated with fixed-step RK4 over
ts = linspace(0, 50, 10000) for 5 initial states (control/certify_segway.py:104-109), through
fiode_amd.odeint (torchdiffeq's 'rk4' with the grid = ts), against the oracle's rk4_on_grid on a
numpy restatement of the same closed loop.  The Segway model / NNController of the reference live
in the empty libs/core submodule: the model is restated (fiode_amd/segway.py), parity unpinned;
the integrator and the LQR start (train_segway.py:31-43) are what this pins."""
import math

import numpy as np
import torch

from oracle import fiode_oracle as O


def _setup():
    from fiode_amd.segway import NNController, Segway, lqr_gain
    torch.manual_seed(0)
    system = Segway()
    K = lqr_gain(system)
    ctrl = NNController(system, 3, 1, 32, K=K)
    with torch.no_grad():                      # a small MLP on top of the LQR start
        for p in ctrl.net.parameters():
            p.mul_(0.1)
    g = torch.Generator().manual_seed(1)
    sizes = torch.tensor([math.pi / 12, 1.5, 1.5])               # train_segway.py:58 sampling box
    x0 = (torch.rand(5, 3, generator=g) * 2 - 1) * sizes
    return system, ctrl, K, x0


def _np_closed_loop(system, ctrl, K):
    W = [m.weight.detach().numpy().astype(np.float32) for m in ctrl.net if isinstance(m, torch.nn.Linear)]
    b = [m.bias.detach().numpy().astype(np.float32) for m in ctrl.net if isinstance(m, torch.nn.Linear)]
    Kn = K.numpy().astype(np.float32)
    f32 = np.float32

    def f(t, x):
        h1 = np.tanh((x @ W[0].T + b[0]).astype(f32)).astype(f32)
        h2 = np.tanh((h1 @ W[1].T + b[1]).astype(f32)).astype(f32)
        u = ((h2 @ W[2].T + b[2]).astype(f32) - (x @ Kn.T).astype(f32)).astype(f32)[:, 0]
        s = np.sin(x[:, 0]).astype(f32)
        dv = ((f32(system.a_v) * s).astype(f32) - (f32(system.d_v) * x[:, 1]).astype(f32)).astype(f32)
        dp = ((f32(system.a_p) * s).astype(f32) - (f32(system.d_p) * x[:, 1]).astype(f32)).astype(f32)
        return np.stack([x[:, 2], (dv + f32(system.b_v) * u).astype(f32),
                         (dp + f32(-system.b_p) * u).astype(f32)], -1).astype(f32)
    return f


def test_lqr_gain_stabilises_linearisation():
    from fiode_amd.segway import Segway, lqr_gain
    system = Segway()
    K = lqr_gain(system)
    F, G = system.jacobian(torch.zeros(1, 3), torch.zeros(1, 1), 0.0)
    assert F.shape == (1, 3, 3) and G.shape == (1, 3, 1)
    A = F[0].numpy() - G[0].numpy() @ K.numpy()
    assert np.linalg.eigvals(F[0].numpy()).real.max() > 0              # the upright plant is unstable
    assert np.linalg.eigvals(A).real.max() < 0                          # the LQR loop is not


def test_segway_simulate_rk4_matches_oracle():
    system, ctrl, K, x0 = _setup()
    ts = np.linspace(0, 50, 10000)
    with torch.no_grad():
        xs, us = system.simulate(x0, ctrl, ts)
    assert xs.shape == (5, 10000, 3) and us.shape == (5, 10000, 1)
    ref = O.rk4_on_grid(_np_closed_loop(system, ctrl, K), x0.numpy(), ts.astype(np.float32))   # [T, B, 3]
    err = float(np.abs(xs.numpy() - ref.transpose(1, 0, 2)).max())
    assert err <= 1e-4, err
    # the closed loop settles: every initial state ends at the same equilibrium (near the goal; the
    # MLP's bias offsets it slightly) and V = |x|^2 ends far below its start
    V = (xs ** 2).sum(-1)
    assert float(V[:, -1].max()) < 1e-4 * float(V[:, 0].min())
    assert float((xs[:, -1] - xs[0, -1]).abs().max()) < 1e-5
    assert torch.isfinite(us).all()
