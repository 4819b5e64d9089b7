"""GPU parity of the fused training step (fiode_lyap_step) and the standalone QP / eval_dot
against the CPU oracle (oracle/fiode_oracle.py).  Runs through the C-ABI (libfiode.so).

Tolerances (fp32): MLP outputs 2e-5 relative to their scale; QP outputs bit-exact given the same
(lower, nominal) inputs; gradients 2e-4 of the gradient's max |entry| (different but equally
valid fp32 summation orders over N rows).  See DESIGN.md "Parity" for why end-to-end gradients
are compared with the QP inputs pinned: the reference decides its backward active set by the sign
of (v - nominal) + mu, which is rounding noise for inactive coordinates.
"""
import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from tests._util import make_params, make_step_inputs

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _ops():
    from fiode_amd import ops, _lib
    return ops, _lib


def _wt(P, dev):
    return {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in
            ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")}


def _run_given(B, S, seed, scale_nominal, dropout=True, kappa=2.0):
    dev = _dev()
    ops, L = _ops()
    P = make_params(seed=seed)
    inp = make_step_inputs(B=B, S=S, seed=seed + 1, dropout=dropout, kappa=kappa)
    cfg = O.DynConfig(scale_nominal=scale_nominal)
    dyn = ops.DynCfg(alpha_1=cfg.alpha_1, alpha_2=cfg.alpha_2, sigma_1=cfg.sigma_1, scale_nominal=scale_nominal,
                     dropout=cfg.dropout)
    masks = None
    mode = L.FIODE_DROPOUT_OFF
    if dropout:
        masks = torch.from_numpy(np.stack([inp.mask1, inp.mask2, inp.lmask1, inp.lmask2])).to(dev)
        mode = L.FIODE_DROPOUT_GIVEN
    sc, gr, dbg = ops.lyap_step(torch.from_numpy(inp.x_feat).to(dev), torch.from_numpy(inp.y).to(dev), _wt(P, dev),
                                dyn, sample_size=S, n_uniform=S, sampler=L.FIODE_SAMPLER_GIVEN, dropout_mode=mode,
                                kappa=kappa, h=torch.from_numpy(inp.h).to(dev), masks=masks, debug=True)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in gr.items()}
    d = {k: v.cpu().numpy() for k, v in dbg.items()}
    return P, inp, cfg, sc.cpu().numpy(), g, d


@pytest.mark.parametrize("B,S,scale_nominal", [(4, 8, True), (4, 8, False), (3, 37, True), (16, 64, False)])
def test_lyap_step_matches_oracle(B, S, scale_nominal):
    P, inp, cfg, sc, g, d = _run_given(B, S, seed=B * 100 + S, scale_nominal=scale_nominal)
    N = B * S
    # 1) MLP + barrier: nominal vs the oracle's own forward
    ref = O.eval_dot(inp.h, np.repeat(O.static_projection(inp.x_feat, P), S, 0), P, cfg, inp.mask1, inp.mask2)
    scale = max(1.0, float(np.abs(ref.nominal).max()))
    err = float(np.abs(d["qp_nominal"][0] - ref.nominal).max())
    assert err <= 2e-5 * scale, err
    # lower = -alpha_1 (exp(sigma_1 h) - 1): one ulp of exp() times alpha_1
    err = float(np.abs(d["qp_lower"] - ref.lower).max())
    assert err <= 2.5e-7 * cfg.alpha_1, err
    # 2) QP on the device's own inputs: bit-exact v and the same global exit iteration
    q = O.qp_forward(d["qp_lower"], d["qp_nominal"][0], cfg.qp_max_iter, cfg.qp_tol)
    assert int(sc[3]) == q.iters
    assert np.array_equal(d["f"], q.v), float(np.abs(d["f"] - q.v).max())
    ql = O.qp_forward(d["qp_lower"], d["qp_nominal"][1], cfg.qp_max_iter, cfg.qp_tol)
    assert int(sc[4]) == ql.iters
    assert np.array_equal(d["f_log"], ql.v), float(np.abs(d["f_log"] - ql.v).max())
    # 3) the whole step with the QP inputs pinned to the device's
    inp.qp_inputs = (d["qp_lower"], d["qp_nominal"][0])
    inp.qp_inputs_log = (d["qp_lower"], d["qp_nominal"][1])
    out = O.lyapunov_step(inp, P, cfg)
    assert np.array_equal(d["V"], out.V)
    assert np.array_equal(d["Vdot"], out.Vdot)
    assert abs(sc[0] - out.loss) <= 1e-5 * max(1.0, abs(out.loss))
    assert int(sc[1]) == out.eff
    assert abs(sc[2] - out.mean_active) <= 1e-7
    gft_ref = out.grads  # noqa: F841
    for k in ("Q3", "b3", "Q2", "b2", "Q1", "b1", "Qx", "bx", "x_feat"):
        a, b = g[k], out.grads[k]
        tol = 2e-4 * max(1e-6, float(np.abs(b).max()))
        assert np.abs(a - b).max() <= tol, (k, float(np.abs(a - b).max()), float(np.abs(b).max()))


def test_lyap_step_full_size_given():
    """BASELINE config shape B=128, S=256 (S1=204 uniform + 52 cone), dropout masks injected."""
    P, inp, cfg, sc, g, d = _run_given(128, 256, seed=7, scale_nominal=True)
    inp.qp_inputs = (d["qp_lower"], d["qp_nominal"][0])
    inp.qp_inputs_log = (d["qp_lower"], d["qp_nominal"][1])
    out = O.lyapunov_step(inp, P, cfg)
    assert int(sc[3]) == out.qp_iters and int(sc[4]) == out.qp_iters_log
    assert abs(sc[0] - out.loss) <= 1e-5 * max(1.0, abs(out.loss))
    assert int(sc[1]) == out.eff
    for k in ("Q3", "b3", "Q2", "b2", "Q1", "b1", "Qx", "bx", "x_feat"):
        a, b = g[k], out.grads[k]
        err = float(np.abs(a - b).max())
        assert err <= 2e-4 * max(1e-6, float(np.abs(b).max())), (k, err)


def test_lyap_step_unpinned_end_to_end():
    """Without pinning: forward scalars agree to fp32 tolerance with the independent oracle."""
    P, inp, cfg, sc, g, d = _run_given(32, 64, seed=3, scale_nominal=True)
    out = O.lyapunov_step(inp, P, cfg)
    assert abs(sc[0] - out.loss) <= 1e-4 * max(1.0, abs(out.loss))
    assert abs(int(sc[1]) - out.eff) <= max(2, out.eff // 500)
    assert np.array_equal(d["V"], out.V)
    err = float(np.abs(d["f"] - out.f).max())
    assert err <= 1e-3, err


def test_lyap_step_philox_sampler_statistics():
    dev = _dev()
    ops, L = _ops()
    P = make_params(seed=5)
    B, S, S1 = 64, 256, 204
    y = torch.randint(0, 10, (B,), device=dev)
    x = torch.randn(B, 10, device=dev)
    sc, gr, dbg = ops.lyap_step(x, y, _wt(P, dev), ops.DynCfg(), sample_size=S, n_uniform=S1, seed=1234, offset=0,
                                debug=True)
    h = dbg["h"].cpu().numpy().reshape(B, S, 10)
    yy = y.cpu().numpy()
    assert np.allclose(h.sum(-1), 1.0, atol=1e-5) and (h >= 0).all()
    # uniform part shared across the batch, Dirichlet(1): E[h_c] = 0.1
    assert np.array_equal(h[0, :S1], h[B - 1, :S1])
    assert abs(h[:, :S1].mean() - 0.1) < 0.01
    # cone part: the label is the argmax
    assert (h[:, S1:].argmax(-1) == yy[:, None]).all()
    # a different offset draws different samples
    _, _, dbg2 = ops.lyap_step(x, y, _wt(P, dev), ops.DynCfg(), sample_size=S, n_uniform=S1, seed=1234, offset=1,
                               debug=True)
    assert not torch.equal(dbg["h"], dbg2["h"])
    assert np.isfinite(sc.cpu().numpy()).all()
    for v in gr.values():
        assert torch.isfinite(v).all()


def test_qp_standalone_bit_exact():
    dev = _dev()
    ops, _ = _ops()
    rng = np.random.default_rng(0)
    for N, scale in ((1, 5.0), (257, 30.0), (5000, 100.0)):
        h = O.uniform_simplex(rng.exponential(1, (N, 10)).astype(np.float32))
        lower = O.barrier_lower(h, O.DynConfig())
        nominal = rng.normal(0, scale, (N, 10)).astype(np.float32)
        v, mu, it = ops.qp_forward(torch.from_numpy(lower).to(dev), torch.from_numpy(nominal).to(dev))
        r = O.qp_forward(lower, nominal)
        assert int(it.item()) == r.iters
        assert np.array_equal(v.cpu().numpy(), r.v)
        assert np.array_equal(mu.cpu().numpy(), r.mu)
        gg = rng.normal(size=(N, 10)).astype(np.float32)
        gl, gn = ops.qp_backward(torch.from_numpy(gg).to(dev), v, mu, torch.from_numpy(lower).to(dev),
                                 torch.from_numpy(nominal).to(dev))
        rl, rn = O.qp_backward(gg, r.v, r.mu, lower, nominal)
        assert np.array_equal(gl.cpu().numpy(), rl) and np.array_equal(gn.cpu().numpy(), rn)


def test_qp_nonconverging_batch_runs_max_iter():
    dev = _dev()
    ops, _ = _ops()
    # huge nominal spread: bisection cannot reach 1e-4 within 30 halvings
    nominal = np.array([[1e8, -1e8, 3, 4, 5, 6, 7, 8, 9, 10]], np.float32)
    lower = np.full((1, 10), -100.0, np.float32)
    v, mu, it = ops.qp_forward(torch.from_numpy(lower).to(dev), torch.from_numpy(nominal).to(dev))
    r = O.qp_forward(lower, nominal)
    assert not r.converged and r.iters == 29 and int(it.item()) == 29
    assert np.array_equal(v.cpu().numpy(), r.v)


@pytest.mark.parametrize("scale_nominal", [True, False])
def test_dyn_eval_matches_oracle(scale_nominal):
    dev = _dev()
    ops, _ = _ops()
    P = make_params(seed=9)
    rng = np.random.default_rng(10)
    B, S = 50, 3
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h = O.uniform_simplex(rng.exponential(1, (B * S, 10)).astype(np.float32))
    cfg = O.DynConfig(scale_nominal=scale_nominal)
    f, it = ops.dyn_eval(torch.from_numpy(h).to(dev), torch.from_numpy(x).to(dev), _wt(P, dev),
                         ops.DynCfg(scale_nominal=scale_nominal), rows_per_image=S)
    ref = O.eval_dot(h, np.repeat(O.static_projection(x, P), S, 0), P, cfg)
    assert abs(int(it.item()) - ref.qp.iters) <= 1
    err = float(np.abs(f.cpu().numpy() - ref.f).max())
    assert err <= 1e-3, err


def test_barrier_projection_function_autograd():
    """FastBarrierProjectionNoUpper drop-in: forward bit-exact, backward = oracle closed form."""
    dev = _dev()
    from fiode_amd.barrier_projection import FastBarrierProjectionNoUpper
    rng = np.random.default_rng(11)
    h = O.uniform_simplex(rng.exponential(1, (700, 10)).astype(np.float32))
    lower = O.barrier_lower(h, O.DynConfig())
    nominal = rng.normal(0, 20, (700, 10)).astype(np.float32)
    proj = FastBarrierProjectionNoUpper(max_iter=30, tol=1e-4)
    lt = torch.from_numpy(lower).to(dev).requires_grad_(True)
    nt = torch.from_numpy(nominal).to(dev).requires_grad_(True)
    v = proj(lt, nt)
    g = rng.normal(size=(700, 10)).astype(np.float32)
    v.backward(torch.from_numpy(g).to(dev))
    r = O.qp_forward(lower, nominal)
    assert np.array_equal(v.detach().cpu().numpy(), r.v)
    gl, gn = O.qp_backward(g, r.v, r.mu, lower, nominal)
    assert np.array_equal(nt.grad.cpu().numpy(), gn) and np.array_equal(lt.grad.cpu().numpy(), gl)


def test_fused_backward_is_bit_reproducible():
    """The fused backward's weight-gradient partials (one fp32 slab per workgroup, summed by
    k_lyap_reduce in a fixed order) make repeated steps on the same inputs bit-identical."""
    dev = _dev()
    ops, L = _ops()
    P = make_params(seed=77)
    B, S = 32, 256
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 10, generator=g).to(dev)
    y = torch.randint(0, 10, (B,), generator=g).to(dev)
    dyn = ops.DynCfg(scale_nominal=True, dropout=0.5)
    runs = []
    for _ in range(3):
        sc, gr, _ = ops.lyap_step(x, y, _wt(P, dev), dyn, sample_size=S, n_uniform=204, seed=3, offset=1)
        torch.cuda.synchronize()
        runs.append((sc.clone(), {k: v.clone() for k, v in gr.items()}))
    for sc, gr in runs[1:]:
        assert torch.equal(sc, runs[0][0])
        for k in gr:
            assert torch.equal(gr[k], runs[0][1][k]), k
