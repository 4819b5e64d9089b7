"""CPU checks of the dopri5 train_ode restatement (oracle/dopri5_train.py): the hand-written reverse
sweep the HIP backward implements (dopri5_adjoint) equals torch autograd through the whole adaptive
solve -- stages, error ratios of accepted and rejected attempts, the step-size controller, the
initial-step selection and the interpolation point -- in float64; and the differentiable forward
takes the oracle's (fiode_oracle.dopri5) step sequence."""
import numpy as np
import pytest
import torch

from oracle import dopri5_train as D
from oracle import fiode_oracle as O
from tests._util import make_params

KEYS = ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")


def _case(B, seed, p=0.5, dtype=torch.float64, E=200):
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.normal(size=(B, 10))).to(dtype)
    h0 = torch.full((B, 10), 0.1, dtype=dtype)
    masks = torch.from_numpy((rng.random((E, 2, B, 128)) >= p).astype(np.uint8)) if p > 0 else None
    W = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dtype).requires_grad_(True) for k in KEYS}
    return P, x, h0, masks, W


@pytest.mark.parametrize("B,seed,sn,rtol", [(16, 1, False, 1e-3), (24, 2, True, 1e-3), (8, 3, False, 3e-4)])
def test_adjoint_sweep_equals_autograd(B, seed, sn, rtol):
    P, x, h0, masks, W = _case(B, seed, E=600)
    g = torch.Generator().manual_seed(seed)
    gout = torch.randn(B, 10, generator=g, dtype=torch.float64)
    yh, st = D.dopri5_train(x, h0, W, masks, rtol=rtol, atol=rtol, scale_nominal=sn, p=0.5)
    (yh * gout).sum().backward()
    ref = {k: W[k].grad.clone() for k in KEYS}
    tr = D.Trace()
    W2 = {k: v.detach().clone().requires_grad_(True) for k, v in W.items()}
    yh2, st2 = D.dopri5_train(x, h0, W2, masks, rtol=rtol, atol=rtol, scale_nominal=sn, p=0.5, leaf_inputs=True,
                              trace=tr)
    assert torch.equal(yh.detach(), yh2.detach()) and st["nfe"] == st2["nfe"]
    print("attempts", [a["accept"] for a in tr.attempts], "nfe", st["nfe"])
    got = D.dopri5_adjoint(tr, gout, W2, rtol=rtol, atol=rtol)
    for k in KEYS:
        scale = float(ref[k].abs().max()) + 1e-30
        err = float((got[k] - ref[k]).abs().max()) / scale
        assert err < 1e-10, (k, err)


def test_controller_gradient_is_present():
    """The step-size controller carries gradient: with the ratio's and dt's paths cut (detached dt) the
    autograd gradient changes -- so the adjoint sweep's controller terms are exercised."""
    P, x, h0, masks, W = _case(16, 4)
    gout = torch.randn(16, 10, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    yh, _ = D.dopri5_train(x, h0, W, masks, scale_nominal=False)
    (yh * gout).sum().backward()
    full = {k: W[k].grad.clone() for k in KEYS}
    tr = D.Trace()
    W2 = {k: v.detach().clone().requires_grad_(True) for k, v in W.items()}
    D.dopri5_train(x, h0, W2, masks, scale_nominal=False, leaf_inputs=True, trace=tr)
    # the same sweep without the scalar (dt / ratio / t / initial-step) terms
    tr_cut = D.Trace()
    tr_cut.Y, tr_cut.K, tr_cut.init = tr.Y, tr.K, dict(tr.init)
    tr_cut.attempts = [dict(a, fmode="hi") for a in tr.attempts]
    cut = D.dopri5_adjoint(tr_cut, gout, W2)
    diff = max(float((cut[k] - full[k]).abs().max()) / (float(full[k].abs().max()) + 1e-30) for k in KEYS)
    assert diff > 1e-6, diff


def test_forward_step_sequence_matches_oracle():
    """Eval mode (no dropout): the differentiable restatement takes fiode_oracle.dopri5's steps and
    reaches its y(t1) (float32 state there, float64 here: to ~1e-5)."""
    P, x, h0, _, W = _case(32, 5, p=0.0)
    cfg = O.DynConfig(scale_nominal=False, dropout=0.0)
    ref, st = O.dopri5(O.make_ode_func(x.numpy().astype(np.float32), P, cfg), h0.numpy().astype(np.float32), 0.0,
                       1.0, rtol=1e-3, atol=1e-3)
    tr = D.Trace()
    yh, s = D.dopri5_train(x, h0, {k: v.detach() for k, v in W.items()}, None, scale_nominal=False, p=0.0, trace=tr)
    assert s["nfe"] == st.nfe
    assert [a["accept"] for a in tr.attempts] == [a for (_, _, a, _) in st.steps]
    assert float((yh - torch.from_numpy(ref).double()).abs().max()) < 1e-4
