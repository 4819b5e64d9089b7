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


def _setup(B, seed, tol, p=0.5, A=64):
    from fiode_amd import _lib as L, ops
    dev = _dev()
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed + 3)
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h0 = np.full((B, 10), 0.1, np.float32)
    mode = L.FIODE_DROPOUT_GIVEN if p > 0 else L.FIODE_DROPOUT_OFF
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.0, mode, method="dopri5", rtol=tol, atol=tol, max_attempts=A)
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


@pytest.mark.parametrize("B,seed,sn,tol", [(64, 3, False, 1e-3), (128, 4, True, 1e-3), (48, 5, False, 3e-4)])
def test_forward_and_gradients_match_float64_autograd(B, seed, sn, tol):
    ops, dev, P, x, h0, cfg, masks, w = _setup(B, seed, tol)
    dyn = ops.DynCfg(scale_nominal=sn, dropout=0.5)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0, s
    sv, nfe, A, acts, mus, accepts = _pins(ops, ws, cfg, s, B)
    assert nfe == 2 + 6 * A and s[4] + s[5] == A
    g = torch.Generator().manual_seed(seed)
    gy = torch.randn(B, 10, generator=g)
    grads, _ = ops.odetrain_backward(gy.to(dev), xt, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    leaves = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).double().requires_grad_(True) for k in KEYS}
    xf = torch.from_numpy(x).double().requires_grad_(True)
    tr = D.Trace()
    yr, info = D.dopri5_train(xf, torch.from_numpy(h0).double(), leaves, torch.from_numpy(masks), 0.0, 1.0, tol, tol,
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
    for k in KEYS + ("x_feat",):
        r = ref[k]
        scale = float(r.abs().max()) + 1e-12
        err = float((grads[k].cpu().double() - r).abs().max()) / scale
        assert err <= 2e-4, (k, err, scale)


def test_attempt_capacity_exhausted_reports_and_poisons():
    """More attempts than max_attempts: status 2 and a NaN y_hat (the loss shows it)."""
    ops, dev, P, x, h0, cfg, masks, w = _setup(32, 6, 1e-6, A=2)
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
    y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                     masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 2 and s[6] == 2 and torch.isnan(y).all()
