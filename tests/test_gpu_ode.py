"""GPU parity of the HIP ODE solves (fiode_odeint) against the oracle's torchdiffeq-0.2.2
restatement (oracle/fiode_oracle.py rk4_fixed_grid / dopri5) on the same dynamics.

Tolerance: 2e-4 absolute on the simplex states.  The solver arithmetic is the same float32
sequence on both sides; the remaining difference is the MLP's float32 accumulation order (MFMA
k-chain vs the oracle's float64 matmul), which can move a stage's batch-global QP exit by one
bisection step (the exit iteration is reported and compared separately).
"""
import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from tests._util import make_params

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _setup(B, seed, scale_nominal):
    from fiode_amd import ops
    dev = _dev()
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed + 1)
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h0 = np.full((B, 10), 0.1, np.float32)
    cfg = O.DynConfig(scale_nominal=scale_nominal)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    return ops, dev, P, x, h0, cfg, w


@pytest.mark.parametrize("B,scale_nominal", [(128, False), (37, True), (300, False)])
def test_rk4_matches_oracle(B, scale_nominal):
    ops, dev, P, x, h0, cfg, w = _setup(B, 10 + B, scale_nominal)
    times = O.linspace32(0.0, 1.0, 2)
    cnt = [0]
    ref, nsteps = O.rk4_fixed_grid(O.make_ode_func(x, P, cfg, cnt), h0, 0.0, 1.0, 0.1, times=times)
    sol, st, dst = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev),
                                  torch.from_numpy(times.astype(np.float64)).to(dev), w,
                                  ops.DynCfg(scale_nominal=scale_nominal, dropout=0.0), method="rk4", step_size=0.1)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0 and s[1] == nsteps == 10 and s[0] == cnt[0] == 40
    err = float(np.abs(sol.cpu().numpy() - ref).max())
    assert err <= 2e-4, err
    assert np.allclose(sol.cpu().numpy()[-1].sum(-1), 1.0, atol=1e-3)


@pytest.mark.parametrize("B,scale_nominal,tol", [(128, False, 1e-3), (64, True, 1e-3), (128, False, 1e-5)])
def test_dopri5_matches_oracle(B, scale_nominal, tol):
    ops, dev, P, x, h0, cfg, w = _setup(B, 20 + B, scale_nominal)
    times = O.linspace32(0.0, 1.0, 2)
    ref, st_ref = O.dopri5(O.make_ode_func(x, P, cfg), h0, 0.0, 1.0, rtol=tol, atol=tol, times=times)
    sol, st, dst = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev),
                                  torch.from_numpy(times.astype(np.float64)).to(dev), w,
                                  ops.DynCfg(scale_nominal=scale_nominal, dropout=0.0), method="dopri5",
                                  rtol=tol, atol=tol)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0
    assert (s[1], s[2]) == (st_ref.n_accept, st_ref.n_reject), (s[:3], st_ref.n_accept, st_ref.n_reject)
    assert s[0] == st_ref.nfe
    err = float(np.abs(sol.cpu().numpy() - ref).max())
    assert err <= 2e-4, err


def test_dopri5_dense_output_many_times():
    ops, dev, P, x, h0, cfg, w = _setup(96, 5, False)
    times = O.linspace32(0.0, 1.0, 9)
    ref, st_ref = O.dopri5(O.make_ode_func(x, P, cfg), h0, 0.0, 1.0, rtol=1e-3, atol=1e-3, times=times)
    sol, st, _ = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev),
                                torch.from_numpy(times.astype(np.float64)).to(dev), w,
                                ops.DynCfg(scale_nominal=False, dropout=0.0), method="dopri5", rtol=1e-3, atol=1e-3)
    torch.cuda.synchronize()
    assert sol.shape == (9, 96, 10)
    err = float(np.abs(sol.cpu().numpy() - ref).max())
    assert err <= 2e-4, err


def test_ivp_forward_through_module():
    """LyapunovLearning.forward (ODELearning.forward, pl_modules.py:322-325) runs the HIP solver."""
    import bench
    dev = _dev()
    mod = bench.build_module(dev)
    mod.eval()
    x = torch.rand(64, 3, 32, 32, device=dev)
    with torch.no_grad():
        out = mod(x)
    stats, _ = mod.dyn_fun.last_solve_stats
    assert out.shape == (64, 10)
    assert torch.isfinite(out).all()
    assert torch.allclose(out.sum(-1), torch.ones(64, device=dev), atol=1e-3)
    assert int(stats[3]) == 0 and int(stats[0]) >= 8


@pytest.mark.parametrize("B", [1024, 4096])
def test_dopri5_large_batch_matches_oracle(B):
    """BASELINE configs[4]'s validation solve size (dopri5 tol 1e-3, models.py:235-241): the solve
    runs one workgroup per 16-row tile (>= B/32 CUs), same NFE / accepted / rejected steps as the
    oracle's torchdiffeq-0.2.2 restatement, states within 2e-4 (as at B=128: with the step sequence
    identical only the MLP's float32 rounding differs)."""
    ops, dev, P, x, h0, cfg, w = _setup(B, 30 + B // 1024, False)
    times = O.linspace32(0.0, 1.0, 2)
    ref, st_ref = O.dopri5(O.make_ode_func(x, P, cfg), h0, 0.0, 1.0, rtol=1e-3, atol=1e-3, times=times)
    sol, st, dst = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev),
                                  torch.from_numpy(times.astype(np.float64)).to(dev), w,
                                  ops.DynCfg(scale_nominal=False, dropout=0.0), method="dopri5", rtol=1e-3, atol=1e-3)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0, s
    assert s[6] >= B // 32 and s[6] * s[7] * 16 >= B, s       # workgroups x tiles x 16 rows cover B
    assert (s[0], s[1], s[2]) == (st_ref.nfe, st_ref.n_accept, st_ref.n_reject), (s[:3], st_ref)
    err = float(np.abs(sol.cpu().numpy() - ref).max())
    assert err <= 2e-4, err


@pytest.mark.parametrize("B,method", [(8192, "dopri5"), (5000, "rk4")])
def test_solve_beyond_resident_capacity(B, method):
    """More tiles than resident workgroups: every workgroup owns several tiles (stats[7] > 1)."""
    ops, dev, P, x, h0, cfg, w = _setup(B, 40, False)
    times = O.linspace32(0.0, 1.0, 3)
    if method == "rk4":
        ref, nsteps = O.rk4_fixed_grid(O.make_ode_func(x, P, cfg), h0, 0.0, 1.0, 0.25, times=times)
        kw = dict(method="rk4", step_size=0.25)
    else:
        ref, st_ref = O.dopri5(O.make_ode_func(x, P, cfg), h0, 0.0, 1.0, rtol=1e-3, atol=1e-3, times=times)
        kw = dict(method="dopri5", rtol=1e-3, atol=1e-3)
    sol, st, _ = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev),
                                torch.from_numpy(times.astype(np.float64)).to(dev), w,
                                ops.DynCfg(scale_nominal=False, dropout=0.0), **kw)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0 and s[7] >= 2 and s[6] * s[7] * 16 >= B, s
    if method == "rk4":
        assert s[1] == nsteps and s[0] == 4 * nsteps
    else:
        assert (s[0], s[1], s[2]) == (st_ref.nfe, st_ref.n_accept, st_ref.n_reject), (s[:3], st_ref)
    err = float(np.abs(sol.cpu().numpy() - ref).max())
    assert err <= 1e-3, err


def test_exchange_timeout_is_reported(monkeypatch):
    """A workgroup that never publishes (FIODE_DEBUG_DROP_PUBLISH test hook: as if it were not
    resident) ends the solve after the bounded spin with status 4, and the module path raises."""
    ops, dev, P, x, h0, cfg, w = _setup(64, 3, False)
    monkeypatch.setenv("FIODE_DEBUG_DROP_PUBLISH", "1")
    times = torch.tensor([0.0, 1.0], dtype=torch.float64, device=dev)
    sol, st, _ = ops.odeint_dyn(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), times, w,
                                ops.DynCfg(scale_nominal=False, dropout=0.0), method="dopri5", rtol=1e-3, atol=1e-3)
    torch.cuda.synchronize()
    assert int(st[3]) == 4
    from fiode_amd.dynamics import OrthoClassDynProjectSimplexLips
    from fiode_amd.odeint import odeint
    dyn = OrthoClassDynProjectSimplexLips(n_hidden=10, activation="ReLU", dropout=0.5, mlp_size=128, kappa=2.0,
                                          kappa_length=0, alpha_1=100.0, alpha_2=20.0, sigma_1=0.02,
                                          scale_nominal=False, x_dim=10, cayley=True).to(dev).eval()
    dyn.static_state = torch.from_numpy(x).to(dev)
    with pytest.raises(RuntimeError, match="timed out"):
        odeint(dyn.ode_forward, (torch.from_numpy(h0).to(dev),), times.float(), rtol=1e-3, atol=1e-3, method="dopri5")
