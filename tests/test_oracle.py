"""CPU known-answer tests pinning the oracle (oracle/fiode_oracle.py) to the reference source
text (SURVEY.md section 4 list) and to the op-for-op torch restatement (oracle/torch_ref.py)."""
import math

import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from oracle import torch_ref as T
from tests._util import make_params, make_step_inputs


# -- schedules / split (sampler_schedulers.py:25-38,72-77; sampler.py:181-192) ------------------

@pytest.mark.parametrize("epoch,expect", [(0, (255, 1)), (10, (255, 1)), (20, (204, 52)),
                                          (35, (127, 129)), (59, (5, 251)), (300, (5, 251))])
def test_mixer_split_table(epoch, expect):
    c = O.cifar_train_mixer(epoch)
    assert abs(c.sum() - 1.0) < 1e-8
    assert tuple(O.split_samples(256, c)) == expect


def test_split_sums_over_epochs():
    for e in range(0, 301):
        s = O.split_samples(256, O.cifar_train_mixer(e))
        assert sum(s) == 256 and min(s) >= 0


# -- samplers -------------------------------------------------------------------------------------

def test_samplers_on_simplex():
    rng = np.random.default_rng(0)
    y = rng.integers(0, 10, 6)
    u = O.uniform_simplex(rng.exponential(1, (50, 10)).astype(np.float32))
    c = O.correct_cone(rng.exponential(1, (6, 40, 10)).astype(np.float32), y)
    d = O.decision_boundary_samples(rng.exponential(1, (6, 40, 9)).astype(np.float32), y)
    for h in (u, c.reshape(-1, 10), d.reshape(-1, 10)):
        assert np.all(h >= 0)
        assert np.allclose(h.sum(-1), 1.0, atol=1e-6)
    assert np.all(np.argmax(c, -1) == y[:, None])
    for b in range(6):
        hy = d[b, :, y[b]]
        wrong = np.delete(d[b], y[b], axis=1)
        assert np.array_equal(hy, wrong.max(-1))


def test_samplers_match_torch_restatement():
    rng = np.random.default_rng(3)
    y = rng.integers(0, 10, 5)
    dr = rng.exponential(1, (5, 17, 10)).astype(np.float32)
    a = O.correct_cone(dr, y)
    b = T.correct_cone(torch.from_numpy(dr.copy()), torch.from_numpy(y)).numpy()
    assert np.allclose(a, b, atol=1e-7)
    du = rng.exponential(1, (33, 10)).astype(np.float32)
    assert np.allclose(O.uniform_simplex(du), T.uniform_simplex(torch.from_numpy(du)).numpy(), atol=1e-7)


# -- Cayley ---------------------------------------------------------------------------------------

@pytest.mark.parametrize("shape", [(128, 10), (128, 128), (10, 128)])
def test_cayley_orthogonal(shape):
    rng = np.random.default_rng(1)
    W = rng.normal(size=shape)
    Q = O.cayley(W)
    if shape[0] >= shape[1]:
        assert np.allclose(Q.T @ Q, np.eye(shape[1]), atol=1e-10)
    else:
        assert np.allclose(Q @ Q.T, np.eye(shape[0]), atol=1e-10)


# -- QP (barrier_projection.py:217-313) ------------------------------------------------------------

def _qp_case(N=200, seed=0, scale=30.0):
    rng = np.random.default_rng(seed)
    h = O.uniform_simplex(rng.exponential(1, (N, 10)).astype(np.float32))
    lower = O.barrier_lower(h, O.DynConfig())
    nominal = (rng.normal(0, scale, (N, 10))).astype(np.float32)
    return lower, nominal


def test_qp_feasible_kkt():
    lower, nominal = _qp_case()
    r = O.qp_forward(lower, nominal)
    assert r.converged
    assert np.all(np.abs(r.v.sum(1)) < 1e-4 + 1e-5)
    assert np.all(r.v >= lower)
    # KKT: v = max(nominal - mu, lower) exactly
    assert np.array_equal(r.v, np.maximum(nominal - r.mu[:, None], lower))


def test_qp_hand_cases():
    # no active bound: v = nominal - mean(nominal)
    nominal = np.array([[1.0, 2.0, 3.0]], np.float32)
    lower = np.full((1, 3), -100.0, np.float32)
    r = O.qp_forward(lower, nominal)
    assert np.allclose(r.v, [[-1, 0, 1]], atol=1e-4)
    # first coordinate at its bound -1: -1 + (1 - mu) + (3 - mu) = 0 -> mu = 1.5
    nominal = np.array([[-10.0, 1.0, 3.0]], np.float32)
    lower = np.full((1, 3), -1.0, np.float32)
    r = O.qp_forward(lower, nominal)
    assert np.allclose(r.v, [[-1, -0.5, 1.5]], atol=1e-4)


def test_qp_global_exit_rule():
    lower, nominal = _qp_case(N=64, seed=4)
    r = O.qp_forward(lower, nominal)
    K = O.global_exit_iteration(r.conv_mask)
    assert K == r.iters
    v2, mu2 = O.qp_run_fixed(lower, nominal, K)
    assert np.array_equal(v2, r.v) and np.array_equal(mu2, r.mu)
    # a single row reaches tol no later than the batch
    for i in range(4):
        ri = O.qp_forward(lower[i:i + 1], nominal[i:i + 1])
        assert ri.iters <= r.iters


def test_qp_matches_torch_restatement():
    lower, nominal = _qp_case(N=300, seed=5)
    r = O.qp_forward(lower, nominal)
    v = T._NoUpperProjection.apply(torch.from_numpy(lower), torch.from_numpy(nominal)).numpy()
    # same iteration count up to residual-summation order; values agree to bisection resolution
    assert np.allclose(r.v, v, atol=2e-4)


def test_qp_backward_vs_dense_and_fd():
    lower, nominal = _qp_case(N=50, seed=6, scale=10.0)
    r = O.qp_forward(lower, nominal)
    g = np.random.default_rng(7).normal(size=nominal.shape).astype(np.float32)
    gl, gn = O.qp_backward(g, r.v, r.mu, lower, nominal)
    # dense-Jacobian torch restatement of the same backward
    lt = torch.from_numpy(lower).requires_grad_(True)
    nt = torch.from_numpy(nominal).requires_grad_(True)
    v = T._NoUpperProjection.apply(lt, nt)
    v.backward(torch.from_numpy(g))
    assert np.allclose(gn, nt.grad.numpy(), atol=1e-6)
    assert np.allclose(gl, lt.grad.numpy(), atol=1e-6)
    # finite differences of the exact projection (float64, tight bisection)
    def proj(nom):
        lo_, hi_ = nom.min(1), (nom - lower).max(1)
        for _ in range(200):
            mu = (lo_ + hi_) / 2
            s = np.maximum(nom - mu[:, None], lower).sum(1)
            lo_ = np.where(s > 0, mu, lo_); hi_ = np.where(s <= 0, mu, hi_)
        return np.maximum(nom - mu[:, None], lower)
    nom64 = nominal.astype(np.float64)
    d = np.random.default_rng(8).normal(size=nominal.shape)
    e = 1e-4
    fd = ((proj(nom64 + e * d) - proj(nom64 - e * d)) / (2 * e) * g).sum()
    an = (gn.astype(np.float64) * d).sum()
    assert abs(fd - an) < 1e-3 * max(1.0, abs(an))


def test_qp_backward_all_active_row():
    # every coordinate at its bound -> g_nominal = 0, g_lower = g (no NaN)
    v = np.array([[-1.0, -2.0]], np.float32)
    lower = v.copy()
    nominal = np.array([[-5.0, -7.0]], np.float32)
    mu = np.array([1.0], np.float32)
    g = np.array([[0.3, -0.2]], np.float32)
    gl, gn = O.qp_backward(g, v, mu, lower, nominal)
    assert np.all(gn == 0) and np.allclose(gl, g)


# -- V and Vdot (lya_cands.py:79-94, pl_modules.py:403-412) ----------------------------------------

def test_vdot_is_directional_derivative():
    rng = np.random.default_rng(2)
    h = O.uniform_simplex(rng.exponential(1, (100, 10)).astype(np.float32)).astype(np.float64)
    y = rng.integers(0, 10, 100)
    f = rng.normal(size=(100, 10))
    V, js = O.decision_boundary_V(h, y)
    Vd = O.vdot(f, y, js)
    e = 1e-7
    Vp, _ = O.decision_boundary_V((h + e * f).astype(np.float64), y)
    def Vexact(hh):
        hw = hh.copy(); hw[np.arange(len(y)), y] = -np.inf
        return 1 + hw.max(1) - hh[np.arange(len(y)), y]
    fd = (Vexact(h + e * f) - Vexact(h)) / e
    assert np.allclose(fd, Vd, atol=1e-4)


# -- full step: closed-form backward vs the reference's autograd/jvp semantics ---------------------

@pytest.mark.parametrize("scale_nominal", [True, False])
@pytest.mark.parametrize("dropout", [True, False])
def test_step_closed_form_matches_autograd(scale_nominal, dropout):
    P = make_params(seed=11)
    inp = make_step_inputs(B=3, S=7, seed=12, dropout=dropout)
    cfg = O.DynConfig(scale_nominal=scale_nominal)
    W = {k: torch.from_numpy(getattr(P, k).copy()) for k in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")}
    tm = lambda a: None if a is None else torch.from_numpy(a.copy())
    stash = {}
    loss, eff, ma, g = T.step_with_grads(
        torch.from_numpy(inp.h.copy()), torch.from_numpy(inp.x_feat.copy()), torch.from_numpy(inp.y),
        inp.S, W, scale_nominal=scale_nominal, kappa=inp.kappa, mask1=tm(inp.mask1), mask2=tm(inp.mask2),
        lmask1=tm(inp.lmask1), lmask2=tm(inp.lmask2), stash=stash)
    # pin the QP inputs (the reference's active-set test is rounding-noise driven, see eval_dot)
    inp.qp_inputs = (stash["lower"].numpy(), stash["nominal"].numpy())
    out = O.lyapunov_step(inp, P, cfg)
    assert abs(loss - out.loss) < 1e-4 * max(1.0, abs(loss))
    assert eff == out.eff
    assert abs(ma - out.mean_active) < 1e-9
    for k in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3", "x_feat"):
        a, b = out.grads[k], g[k].numpy()
        tol = 1e-4 * max(1e-3, float(np.abs(b).max()))
        assert np.allclose(a, b, atol=tol), (k, np.abs(a - b).max(), np.abs(b).max())


# -- ODE solvers (torchdiffeq 0.2.2 semantics) ------------------------------------------------------

def test_rk4_38_exact_on_cubic():
    # dy/dt = 3t^2 + 2t + 1 (time-only): 3/8 rule is exact on cubics
    func = lambda t, y: np.full_like(y, 3 * t * t + 2 * t + 1, dtype=np.float32)
    y, nsteps = O.rk4_fixed_grid(func, np.zeros((2, 3), np.float32), 0.0, 1.0, 0.1)
    assert nsteps == 10
    assert np.allclose(y, 3.0, atol=1e-5)


def test_rk4_grid_rule():
    calls = []
    func = lambda t, y: (calls.append(t), np.zeros_like(y))[1]
    _, nsteps = O.rk4_fixed_grid(func, np.zeros((1, 1), np.float32), 0.0, 1.0, 0.3)
    assert nsteps == 4   # ceil(1/0.3 + 1) = 5 points, last snapped to 1.0


def test_dopri5_linear_ode():
    A = -np.linspace(0.5, 3.0, 10).astype(np.float32)
    func = lambda t, y: (y * A).astype(np.float32)
    y0 = np.ones((4, 10), np.float32)
    y, st = O.dopri5(func, y0, 0.0, 1.0, rtol=1e-6, atol=1e-6)
    assert np.allclose(y, np.exp(A)[None] * y0, rtol=1e-4, atol=1e-5)
    assert st.nfe == 2 + 6 * (st.n_accept + st.n_reject)


def test_dopri5_on_dynamics_matches_fine_reference():
    P = make_params(seed=21)
    cfg = O.DynConfig(scale_nominal=False)
    rng = np.random.default_rng(22)
    x = rng.normal(size=(6, 10)).astype(np.float32)
    h0 = np.full((6, 10), 0.1, np.float32)
    func = O.make_ode_func(x, P, cfg)
    y, st = O.dopri5(func, h0, 0.0, 1.0, rtol=1e-3, atol=1e-3)
    yf, _ = O.rk4_fixed_grid(func, h0, 0.0, 1.0, 0.002)
    assert np.allclose(y.sum(1), 1.0, atol=1e-3)
    assert np.abs(y - yf).max() < 2e-2


# -- certification grid (eval_utils.py:31-89) -------------------------------------------------------

def test_grid_count_G_10_40():
    assert O.db_count_table(10, 40)[40][10] == 41_320_837


@pytest.mark.parametrize("n,T", [(3, 6), (4, 8), (5, 10), (10, 4)])
def test_grid_order_and_unrank(n, T):
    import itertools
    g = O.db_grid_rows(n, T)
    f = O.db_count_table(n, T)
    assert g.shape[0] == f[T][n]
    brute = {v for v in itertools.product(range(T + 1), repeat=n) if sum(v) == T and v[0] == max(v[1:])}
    assert set(map(tuple, g.tolist())) == brute
    assert len(brute) == g.shape[0]                 # no duplicates
    for r in range(g.shape[0]):
        assert O.db_unrank(r, n, T, f) == g[r].tolist()


def test_certify_batches_rule():
    assert O.certify_batches(41_320_837, 10)[-1] == (41_320_830, 41_320_837)
    assert len(O.certify_batches(41_320_837, 10)) == 11
    assert O.certify_batches(20, 10) == [(2 * i, 2 * i + 2) for i in range(10)]


def test_rk4_train_oracle_matches_torch_ref_forward():
    """The numpy train-mode RK4 (fiode_oracle.rk4_train) and the autograd restatement
    (torch_ref.ode_train_loss) agree on y(t1) with the same dropout masks."""
    import torch
    from oracle import torch_ref as T
    P = make_params(3)
    cfg = O.DynConfig(scale_nominal=True)
    rng = np.random.default_rng(0)
    B = 16
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h0 = np.full((B, 10), 0.1, np.float32)
    masks = (rng.random((16, 2, B, 128)) < 0.5).astype(np.uint8)
    y, recs = O.rk4_train(x, h0, P, cfg, 0.0, 1.0, 0.25, masks, 0.5)
    assert len(recs) == 16
    W = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))) for k in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")}
    loss, yy = T.ode_train_loss(torch.from_numpy(x), torch.from_numpy(h0), torch.from_numpy(rng.integers(0, 10, B)),
                                W, torch.from_numpy(masks), 0.0, 1.0, 0.25)
    assert np.abs(yy.numpy() - y).max() < 1e-4
    assert np.allclose(y.sum(-1), 1.0, atol=1e-3)


def test_pinned_active_set_backward_equals_reference_backward():
    """torch_ref._PinnedActiveSet with the projection's own active set = _NoUpperProjection."""
    import torch
    from oracle import torch_ref as T
    rng = np.random.default_rng(4)
    h = O.uniform_simplex(rng.exponential(1, (50, 10)).astype(np.float32))
    lower = torch.from_numpy(O.barrier_lower(h, O.DynConfig()))
    nom = torch.from_numpy(rng.normal(0, 10, (50, 10)).astype(np.float32))
    g = torch.from_numpy(rng.normal(size=(50, 10)).astype(np.float32))
    a1, n1 = lower.clone().requires_grad_(True), nom.clone().requires_grad_(True)
    v = T._NoUpperProjection.apply(a1, n1)
    (v * g).sum().backward()
    r = O.qp_forward(lower.numpy(), nom.numpy())
    act = torch.from_numpy(((r.v - nom.numpy()) + r.mu[:, None]) > 0)
    a2, n2 = lower.clone().requires_grad_(True), nom.clone().requires_grad_(True)
    v2 = T._PinnedActiveSet.apply(a2, n2, act)
    (v2 * g).sum().backward()
    assert torch.allclose(a1.grad, a2.grad, atol=1e-6) and torch.allclose(n1.grad, n2.grad, atol=1e-6)
