"""TrajectorySampler (sampler.py:156-166).

CPU: the fixed-grid output rule used to turn the train-mode solve's grid states into the
trajectory at linspace(0, t_max, n) equals torchdiffeq 0.2.2's FixedGridODESolver rule as restated in
odeint._odeint_torch (same float32 interval choice, exact-hit picks, lerp).
GPU: the fused step with sampler TRAJECTORY reads the trajectory rows where the reference's
CompositeSampler puts them (after the Uniform rows, per image), and equals the same step run with
the assembled samples given (GIVEN) -- bit for bit; the eval-mode trajectory is fiode_odeint's
solution at the n times; the train-mode trajectory starts at h0, ends at the solve's y(t1) and
interpolates the solve's grid states.
"""
import pathlib
import sys

import numpy as np
import pytest
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "fi-ode_amd"))


@pytest.mark.parametrize("n,step", [(2, 0.1), (11, 0.1), (52, 0.1), (100, 0.07), (7, 0.25)])
def test_fixed_grid_interp_plan_matches_torch_rule(n, step):
    from fiode_amd.odeint import _odeint_torch, _rk4_grid
    from fiode_amd.sampling import fixed_grid_interp_plan
    t = torch.linspace(0.0, 1.0, n)
    grid = _rk4_grid(t[0], t[-1], step, torch.float32)
    # a right-hand side whose rk4 steps are exact (f = const) makes the grid states known: y(t) = y0 + c t
    y0 = torch.tensor([[0.3, -1.0, 2.0]])
    c = torch.tensor([[1.5, 0.25, -3.0]])
    ref = _odeint_torch(lambda tt, yy: c.expand_as(yy), y0, t, 0, 0, "rk4", {"step_size": step})
    # grid states exactly as the solver produced them
    states = [y0]
    y = y0
    for a, b in zip(grid[:-1], grid[1:]):
        dt = b - a
        k1 = c; k2 = c; k3 = c; k4 = c
        y = y + (k1 + 3 * (k2 + k3) + k4) * dt * 0.125
        states.append(y)
    G = torch.stack(states, dim=1)               # [1, niters, 3]
    k, slope, pick = fixed_grid_interp_plan(grid, t)
    kt = torch.from_numpy(k)
    ya, yb = G[:, kt], G[:, kt + 1]
    out = ya + torch.from_numpy(slope)[None, :, None] * (yb - ya)
    p = torch.from_numpy(pick)[None, :, None]
    out = torch.where(p == 1, ya, torch.where(p == 2, yb, out))
    assert torch.equal(out[0], ref[:, 0]), (out[0] - ref[:, 0]).abs().max()


def test_kernel_plan_trajectory_kinds():
    from fiode_amd import _lib as L
    from fiode_amd.sampling import CompositeSampler, TrajectorySampler, UniformSimplexSampling
    cs = CompositeSampler((10,), [UniformSimplexSampling(), TrajectorySampler()])
    assert cs.kernel_plan(256, [0.8, 0.2]) == (L.FIODE_SAMPLER_TRAJECTORY, 204)
    assert CompositeSampler((10,), [TrajectorySampler()]).kernel_plan(64, [1.0]) == (L.FIODE_SAMPLER_TRAJECTORY, 0)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _traj_module(dev, train_ode_solver="rk4", tol=0.1):
    import bench
    from fiode_amd.sampling import CompositeSampler, TrajectorySampler, UniformSimplexSampling
    mod = bench.build_module(dev, seed=0, train_ode=False)
    mod.sampler = CompositeSampler((10,), [UniformSimplexSampling(), TrajectorySampler()])
    mod.train_ode_solver, mod.train_ode_tol = train_ode_solver, tol
    return mod


@pytest.mark.gpu
@pytest.mark.parametrize("training", [False, True])
def test_fused_step_trajectory_equals_given(training):
    from fiode_amd import _lib as L, ops
    dev = _gpu()
    mod = _traj_module(dev)
    mod.train(training)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(16, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (16,), generator=g).to(dev)
    with torch.no_grad():
        static, _ = mod.init_coordinates(x, mod.dyn_fun)
    static = static.float().contiguous()
    S = mod.h_sample_size
    S1 = mod.sampler.kernel_plan(S, mod.sampler_scheduler.get_mixer_coefficients(mod.current_epoch))[1]
    traj = mod.sampler.samplers[1].trajectory(mod, static, S - S1)
    assert traj.shape == (16, S - S1, 10)
    w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
    kw = dict(sample_size=S, n_uniform=S1, dropout_mode=L.FIODE_DROPOUT_OFF, kappa=2.0, seed=7, offset=3, debug=True)
    sc_t, gr_t, dbg_t = ops.lyap_step(static, y, w, mod.dyn_fun.dyn_cfg(), sampler=L.FIODE_SAMPLER_TRAJECTORY,
                                      h=traj, **kw)
    sc_t, gr_t = sc_t.clone(), {k: v.clone() for k, v in gr_t.items()}
    h_all = dbg_t["h"].view(16, S, 10)
    assert torch.equal(h_all[:, S1:], traj)                     # trajectory rows after the Uniform rows
    assert torch.equal(h_all[0, :S1], h_all[5, :S1])           # Uniform rows shared over the batch
    sc_g, gr_g, _ = ops.lyap_step(static, y, w, mod.dyn_fun.dyn_cfg(), sampler=L.FIODE_SAMPLER_GIVEN,
                                  h=dbg_t["h"].clone(), **kw)
    torch.cuda.synchronize()
    assert torch.equal(sc_t, sc_g)
    for k in gr_t:
        assert torch.equal(gr_t[k], gr_g[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("solver,tol", [("rk4", 0.1), ("dopri5", 1e-3)])
def test_eval_trajectory_is_odeint_solution(solver, tol):
    from fiode_amd import ops
    dev = _gpu()
    mod = _traj_module(dev, solver, tol).eval()
    g = torch.Generator().manual_seed(4)
    x = torch.rand(8, 3, 32, 32, generator=g).to(dev)
    with torch.no_grad():
        static, _ = mod.init_coordinates(x, mod.dyn_fun)
        traj = mod.sampler.samplers[1].trajectory(mod, static.float(), 52)
        ref = mod.model(x, ts=torch.linspace(0.0, 1.0, 52, device=dev), int_params=mod.train_solver_params,
                        return_traj=True)                      # the reference's call (sampler.py:163-165)
        w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
        p = mod.train_solver_params
        sol, _, _ = ops.odeint_dyn(static.float().contiguous(), mod.init_coordinates.h0_0[None].expand(8, -1).contiguous(),
                                   torch.linspace(0.0, 1.0, 52).to(dev, torch.float64), w, mod.dyn_fun.dyn_cfg(),
                                   method=p["method"], rtol=p.get("rtol", 0.0), atol=p.get("atol", 0.0),
                                   step_size=p.get("options", {}).get("step_size"))
    torch.cuda.synchronize()
    assert torch.equal(traj, sol.transpose(0, 1))               # the solve at the n times, transposed
    # the reference's call recomputes the backbone features (last-bit differences can move a QP exit):
    # the ODE tolerance of tests/test_gpu_ode.py
    err = float((traj - ref.transpose(0, 1)).abs().max())
    assert err <= 2e-4, err
    assert torch.allclose(traj.sum(-1), torch.ones_like(traj.sum(-1)), atol=1e-3)


@pytest.mark.gpu
def test_train_mode_trajectory_interpolates_solve():
    from fiode_amd import _lib as L, ops
    from fiode_amd.odeint import _rk4_grid
    dev = _gpu()
    mod = _traj_module(dev).train()
    g = torch.Generator().manual_seed(6)
    x = torch.rand(8, 3, 32, 32, generator=g).to(dev)
    with torch.no_grad():
        static, _ = mod.init_coordinates(x, mod.dyn_fun)
    static = static.float().contiguous()
    ts = mod.sampler.samplers[1]
    traj = ts.trajectory(mod, static, 31)
    # the same train-mode solve (same Philox seed / offset) run directly
    w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
    cfg = ops.odetrain_config(8, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=mod.seed ^ ts.TRAJ_SEED_SALT,
                              offset=mod._rng_offset)
    h0 = mod.init_coordinates.h0_0[None].expand(8, -1).float().contiguous()
    y1, _, ws = ops.odetrain_forward(static, h0, w, mod.dyn_fun.dyn_cfg(), cfg)
    G = torch.cat([ops.odetrain_saved(ws, cfg)["h"][:, 0::4], y1[:, None]], 1)
    torch.cuda.synchronize()
    assert torch.equal(traj[:, 0], h0) and torch.equal(traj[:, -1], y1)
    grid = _rk4_grid(torch.tensor(0.0), torch.tensor(1.0), 0.1, torch.float32).numpy()
    t = torch.linspace(0.0, 1.0, 31).numpy()
    Gc, Tc = G.cpu().numpy(), traj.cpu().numpy()
    for j in range(1, 31):
        i = int(np.searchsorted(grid, t[j], side="left")) - 1
        i = max(i, 0)
        lam = (t[j] - grid[i]) / (grid[i + 1] - grid[i])
        np.testing.assert_allclose(Tc[:, j], Gc[:, i] + lam * (Gc[:, i + 1] - Gc[:, i]), atol=1e-6)
    # dropout is on: the trajectory differs from the eval-mode solve
    ev = _traj_module(dev).eval()
    ev.load_state_dict(mod.state_dict())
    assert not torch.equal(ev.sampler.samplers[1].trajectory(ev, static, 31), traj)


@pytest.mark.gpu
def test_compute_loss_with_trajectory_sampler():
    dev = _gpu()
    mod = _traj_module(dev).train()
    g = torch.Generator().manual_seed(8)
    x = torch.rand(16, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (16,), generator=g).to(dev)
    loss = mod.compute_loss(x, y, 16, "relu")
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in mod.parameters() if p.grad is not None)
    assert mod.dyn_fun.mlp_to_mlp.weight.grad.abs().sum() > 0
