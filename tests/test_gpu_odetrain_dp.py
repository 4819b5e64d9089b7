"""GPU parity of the differentiable train_ode solve with adaptive dopri5 (cifar_train.yaml:30,32:
train_ode_solver dopri5, train_ode_tol 1e-3; pl_modules.py:490-500, models.py:235-241; direct
backprop, use_adjoint False at pl_modules.py:303) -- fiode_odetrain_forward / _backward with
method FIODE_ODE_DOPRI5.

* dropout off: the forward takes the eval solve's (fiode_odeint dopri5) steps -- same NFE, accept /
  reject sequence -- and reaches its y(t1) bit for bit on 16-row tiles (B > 1,024: the same MLP / QP
  kernels), within 1e-4 on 4-row tiles (B <= 1,024: the MLP sums in another order, which moves
  each QP solution within its bisection resolution);
* train mode (given dropout masks): every eval's stage input and the output agree with the float64
  restatement oracle/dopri5_train.py run at the device's linearisation points (QP active sets, exit
  mu and accept decisions pinned) -- same NFE and accept / reject sequence;
* gradients (all eight weight tensors and x_feat) within 2e-4 of each tensor's max of float64
  torch autograd through that restatement: stages, error ratios of accepted and rejected attempts,
  the step-size controller, the initial step and the interpolation point."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import dopri5_train as D
from tests._util import make_params

pytestmark = pytest.mark.gpu
KEYS = ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _setup(B, seed, tol, p=0.5, A=64, t1=1.0):
    from fiode_amd import _lib as L, ops
    dev = _dev()
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed + 3)
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h0 = np.full((B, 10), 0.1, np.float32)
    mode = L.FIODE_DROPOUT_GIVEN if p > 0 else L.FIODE_DROPOUT_OFF
    cfg = ops.odetrain_config(B, 0.0, t1, 0.0, mode, method="dopri5", rtol=tol, atol=tol, max_attempts=A)
    E = ops.odetrain_evals(cfg)
    assert E == 2 + 6 * A
    masks = (rng.random((E, 2, B, 128)) >= p).astype(np.uint8) if p > 0 else None
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in KEYS}
    return ops, dev, P, x, h0, cfg, masks, w


@pytest.mark.parametrize("B,seed,sn", [(64, 1, False), (128, 2, True), (1040, 3, False)])
def test_dropout_off_equals_eval_solve(B, seed, sn):
    ops, dev, P, x, h0, cfg, _, w = _setup(B, seed, 1e-3, p=0.0)
    dyn = ops.DynCfg(scale_nominal=sn, dropout=0.0)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg)
    sol, est, _ = ops.odeint_dyn(xt, h0t, torch.tensor([0.0, 1.0], dtype=torch.float64, device=dev), w, dyn,
                                 method="dopri5", rtol=1e-3, atol=1e-3)
    torch.cuda.synchronize()
    s, e = st.cpu().numpy(), est.cpu().numpy()
    assert s[3] == 0 and e[3] == 0, (s, e)
    assert (s[0], s[4], s[5]) == (e[0], e[1], e[2]), (s, e)
    if B > 1024:              # 16-row tiles: the eval solve's MLP and QP kernels
        assert torch.equal(y, sol[-1])
    else:                     # 4-row tiles (tile4.h): the same solve, MLP sums in another order
        assert float((y - sol[-1]).abs().max()) <= 1e-4     # QP bisection resolution (tol 1e-4)


def _pins(ops, ws, cfg, st, B):
    sv = ops.odetrain_saved(ws, cfg)
    nfe, A = int(st[0]), int(st[6])
    act = ((sv["v"] - sv["nominal"]) + sv["mu"][..., None] > 0).cpu()          # [B,E,C]
    acts = [act[:, e] for e in range(nfe)]
    mus = [sv["mu"][:, e].double().cpu() for e in range(nfe)]
    accepts = [bool(a) for a in sv["attempts"][:A, 3].cpu().numpy()]
    return sv, nfe, A, acts, mus, accepts


def _check_grads(grads, ref, tol=2e-4):
    for k in KEYS + ("x_feat",):
        r = ref[k]
        scale = float(r.abs().max()) + 1e-12
        err = float((grads[k].cpu().double() - r).abs().max()) / scale
        assert err <= tol, (k, err, scale)


# (64, 7, t1 = 0.05, tol 0.1): the solve accepts its FIRST attempt (nfe 8 = 2 initial-step evals +
# 6 stages): the forward makes 3 reduction exchanges, so a backward that restarted the exchange
# epochs would meet the forward's stale tags (round-3 review) -- its gradients must still match.
@pytest.mark.parametrize("B,seed,sn,tol,t1", [(64, 3, False, 1e-3, 1.0), (128, 4, True, 1e-3, 1.0),
                                              (48, 5, False, 3e-4, 1.0), (64, 7, False, 0.1, 0.05)])
def test_forward_and_gradients_match_float64_autograd(B, seed, sn, tol, t1):
    ops, dev, P, x, h0, cfg, masks, w = _setup(B, seed, tol, t1=t1)
    dyn = ops.DynCfg(scale_nominal=sn, dropout=0.5)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0, s
    sv, nfe, A, acts, mus, accepts = _pins(ops, ws, cfg, s, B)
    assert nfe == 2 + 6 * A and s[4] + s[5] == A
    if t1 < 1.0:
        assert A == 1 and nfe == 8, (A, nfe)
    g = torch.Generator().manual_seed(seed)
    gy = torch.randn(B, 10, generator=g)
    grads, _ = ops.odetrain_backward(gy.to(dev), xt, w, dyn, cfg, ws)
    # a second sweep on the same workspace (its exchanges continue the epoch sequence): the same
    # gradients, bit for bit
    grads2, _ = ops.odetrain_backward(gy.to(dev), xt, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    for k in KEYS + ("x_feat",):
        assert torch.equal(grads[k], grads2[k]), k
    assert int(ops.odetrain_status_word(ws, cfg)[0]) == 0
    leaves = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).double().requires_grad_(True) for k in KEYS}
    xf = torch.from_numpy(x).double().requires_grad_(True)
    tr = D.Trace()
    yr, info = D.dopri5_train(xf, torch.from_numpy(h0).double(), leaves, torch.from_numpy(masks), 0.0, t1, tol, tol,
                              scale_nominal=sn, p=0.5, acts=acts, mus=mus, accepts=accepts, trace=tr)
    assert info["nfe"] == nfe
    # every eval's stage input, then the output
    hin = sv["h"][:, :nfe].cpu().double()
    herr = max(float((hin[:, e] - tr.Y[e].detach()).abs().max()) for e in range(nfe))
    assert herr <= 2e-4, herr
    assert float((y.cpu().double() - yr.detach()).abs().max()) <= 2e-4
    (yr * gy.double()).sum().backward()
    ref = {k: leaves[k].grad for k in KEYS}
    ref["x_feat"] = xf.grad
    _check_grads(grads, ref)


def test_attempt_capacity_exhausted_reports_and_poisons():
    """More attempts than max_attempts: status 2 and a NaN y_hat (the loss shows it)."""
    ops, dev, P, x, h0, cfg, masks, w = _setup(32, 6, 1e-6, A=2)
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
    y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                     masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 2 and s[6] == 2 and torch.isnan(y).all()
    assert int(ops.odetrain_status_word(ws, cfg)[0]) == 2


def test_lazy_keep_words_equal_drawn_up_front():
    """Philox dropout at p = 0.5 (the YAML's): the dopri5 forward draws each eval's keep words
    itself and saves them (k_ot_masks no longer draws the whole attempt capacity up front).  They
    are the words k_ot_masks draws (same Philox stream per (eval, set, row)): the first evals' words
    of a dopri5 solve equal those an rk4 solve of the same seed and offset gets from k_ot_masks."""
    from fiode_amd import _lib as L, ops
    dev = _dev()
    B = 64
    P = make_params(seed=9)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in KEYS}
    xt = torch.randn(B, 10, generator=torch.Generator().manual_seed(9)).to(dev)
    h0 = torch.full((B, 10), 0.1, device=dev)
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
    kw, nfe = {}, {}
    for method in ("dopri5", "rk4"):
        cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=11, offset=3, method=method,
                                  rtol=1e-3, atol=1e-3, max_attempts=64)
        y, st, ws = ops.odetrain_forward(xt, h0, w, dyn, cfg)
        torch.cuda.synchronize()
        assert int(st[3]) == 0 and bool(torch.isfinite(y).all())
        kw[method], nfe[method] = ops.odetrain_saved(ws, cfg)["keep_words"].clone(), int(st[0])
    n = min(nfe["dopri5"], nfe["rk4"])
    assert n >= 8
    assert torch.equal(kw["dopri5"][:n], kw["rk4"][:n])
    assert int(torch.count_nonzero(kw["dopri5"][:n])) > 0
