"""GPU parity of the differentiable train-mode RK4 solve (fiode_odetrain_forward / _backward,
the train_ode branch of pl_modules.py:490-500) against the oracle (numpy forward,
oracle.fiode_oracle.rk4_train) and torch autograd through the reference-order RK4 stages
(oracle.torch_ref.ode_train_loss) with the same dropout masks.

Tolerances: forward 2e-4 absolute on the simplex state (MLP accumulation order can move a
stage's batch-global QP exit by one bisection step, as in test_gpu_ode).  Gradients: 2e-4 of each
tensor's max-abs against float64 torch autograd through the reference-order RK4 stages, evaluated
at the device's linearisation points: the QP active sets (the reference's active-set test is
float32 rounding noise on inactive coordinates) and each eval's exit mu are pinned to the
device's, so the remaining difference is the device's float32 rounding over 40 stage VJPs."""
import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from tests._util import make_params

pytestmark = pytest.mark.gpu
KEYS = ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _case(B, step, scale_nominal, seed, p=0.5):
    from fiode_amd import _lib as L, ops
    dev = _dev()
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed + 7)
    x = rng.normal(size=(B, 10)).astype(np.float32)
    h0 = np.full((B, 10), 0.1, np.float32)
    labels = rng.integers(0, 10, B)
    cfg = ops.odetrain_config(B, 0.0, 1.0, step, L.FIODE_DROPOUT_GIVEN if p > 0 else L.FIODE_DROPOUT_OFF)
    E = ops.odetrain_evals(cfg)
    masks = (rng.random((E, 2, B, 128)) >= p).astype(np.uint8) if p > 0 else None
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in KEYS}
    dyn = ops.DynCfg(scale_nominal=scale_nominal, dropout=p)
    return ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn


@pytest.mark.parametrize("B,step,scale_nominal", [(64, 0.25, True), (128, 0.1, False), (37, 0.3, True)])
def test_forward_matches_oracle(B, step, scale_nominal):
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(B, step, scale_nominal, 100 + B)
    ref, recs = O.rk4_train(x, h0, P, O.DynConfig(scale_nominal=scale_nominal), 0.0, 1.0, step, masks, 0.5)
    assert len(recs) == E
    y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                     masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[0] == E and s[1] == E // 4 and s[3] == 0
    err = float(np.abs(y.cpu().numpy() - ref).max())
    assert err <= 2e-4, err
    sv = ops.odetrain_saved(ws, cfg)
    herr = max(float(np.abs(sv["h"][:, e].cpu().numpy() - recs[e][0]).max()) for e in range(E))
    assert herr <= 2e-4, herr


@pytest.mark.parametrize("B,step,scale_nominal", [(64, 0.25, True), (128, 0.1, False), (48, 0.5, False)])
def test_backward_matches_torch_autograd(B, step, scale_nominal):
    from oracle import torch_ref as T
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(B, step, scale_nominal, 200 + B)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=torch.from_numpy(masks).to(dev))
    yd = y.detach().clone().requires_grad_(True)
    lab = torch.from_numpy(labels).to(dev)
    torch.nn.functional.nll_loss(torch.log(yd), lab).backward()
    grads, _ = ops.odetrain_backward(yd.grad, xt, w, dyn, cfg, ws)
    sv = ops.odetrain_saved(ws, cfg)
    act = ((sv["v"] - sv["nominal"]) + sv["mu"][..., None] > 0).cpu()          # [B,E,C]
    acts = [act[:, e] for e in range(E)]
    mus = [sv["mu"][:, e].double().cpu() for e in range(E)]
    # float64 autograd at the device's linearisation points (QP active sets and exit mu pinned)
    leaves = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).double().requires_grad_(True) for k in KEYS}
    xf = torch.from_numpy(x).double().requires_grad_(True)
    loss, yy = T.ode_train_loss(xf, torch.from_numpy(h0).double(), torch.from_numpy(labels), leaves,
                                torch.from_numpy(masks), 0.0, 1.0, step, scale_nominal=scale_nominal, p=0.5, acts=acts,
                                mus=mus)
    loss.backward()
    ref = {k: leaves[k].grad for k in KEYS}
    ref["x_feat"] = xf.grad
    for k in KEYS + ("x_feat",):
        g = grads[k].cpu().double()
        r = ref[k]
        scale = float(r.abs().max()) + 1e-12
        err = float((g - r).abs().max()) / scale
        assert err <= 2e-4, (k, err, scale)


def test_philox_masks_fresh_per_offset():
    from fiode_amd import _lib as L
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(64, 0.25, True, 5)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    outs = []
    for off in (0, 0, 1):
        c = ops.odetrain_config(64, 0.0, 1.0, 0.25, L.FIODE_DROPOUT_PHILOX, seed=9, offset=off)
        y, _, _ = ops.odetrain_forward(xt, h0t, w, dyn, c)
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1]) and not torch.equal(outs[0], outs[2])
    assert torch.isfinite(outs[2]).all()
    assert torch.allclose(outs[2].sum(-1), torch.ones(64), atol=1e-3)


def test_module_train_ode_loss_mix():
    """compute_loss with train_ode: loss = (1-p) lyapunov + p nll(log y_hat), p = min(.98, (epoch -
    train_ode_epoch)/50) (pl_modules.py:490-500); gradients reach the backbone and the dynamics."""
    import bench
    dev = _dev()
    mod = bench.build_module(dev, seed=0, train_ode=True)
    x = torch.rand(16, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    loss = mod.compute_loss(x, y, 16, "relu")
    lyap = float(mod.last_plan["scalars"][0])
    lode = float(mod.logged["loss_ode"])
    p = min(0.98, (bench.EPOCH - bench.TRAIN_ODE_EPOCH) / 50.0)
    assert abs(float(loss) - ((1 - p) * lyap + p * lode)) < 1e-5
    loss.backward()
    for name, prm in mod.named_parameters():
        if prm.requires_grad:
            assert prm.grad is not None and torch.isfinite(prm.grad).all(), name
    torch.cuda.synchronize()
    s = mod.last_ode_plan["stats"].cpu()
    assert int(s[0]) == 40 and int(s[1]) == 10


@pytest.mark.parametrize("reuse", [True, False])
def test_fused_loss_node_equals_three_nodes(reuse):
    """LyapODELossFn (the configs[1] loss as one autograd node) = the three-node graph
    (LyapunovLossFn + ODETrainFn + ODELossMixFn): same loss and the same gradients bit for bit --
    the node sums ode + lyap * ((1 - p) go) exactly as autograd's accumulation does, with the same
    Philox draws (same seed / offset) and the solve on its side stream in both."""
    import bench
    from fiode_amd import lyapunov as LY
    dev = _dev()
    x = torch.rand(32, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    yb = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(6))
    out = {}
    LY.DYN_WGRAD_SIDE = False          # the one-call backward (the split one: the test below)
    try:
        for variant in ("fused", "three"):
            mod = bench.build_module(dev, seed=0, train_ode=True)
            mod.parallel_cayley = False
            mod.ode_reuse_features = reuse
            mod.fused_ode_loss = variant != "three"
            mod._rng_offset = 0
            loss = mod.compute_loss(x, yb, 32, "relu")
            loss.backward()
            torch.cuda.synchronize()
            out[variant] = (loss.detach().clone(), float(mod.logged["loss_ode"]),
                            {n: p.grad.detach().clone() for n, p in mod.named_parameters() if p.requires_grad})
    finally:
        LY.DYN_WGRAD_SIDE = True
    lb, ob, gb = out["three"]
    la, oa, ga = out["fused"]
    assert torch.equal(la, lb) and oa == ob
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n


@pytest.mark.parametrize("reuse", [True, False])
def test_dynamics_weight_grad_node_matches_one_call(reuse):
    """The dynamics weights' gradients as their own side-stream node (_DynWeightTapFn: the solve's
    backward split into fiode_odetrain_backward_x + _weights) against the one-call backward: the same
    loss, the dynamics parameters' gradients bit for bit, the backbone's within float32 rounding
    (dL/dx_feat is the same sum in another order, test_split_backward_entry_points_equal_one_call)."""
    import bench
    from fiode_amd import lyapunov as LY
    dev = _dev()
    x = torch.rand(32, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    yb = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(6))
    out = {}
    try:
        for side in (True, False):
            LY.DYN_WGRAD_SIDE = side
            mod = bench.build_module(dev, seed=0, train_ode=True)
            mod.ode_reuse_features = reuse
            mod._rng_offset = 0
            loss = mod.compute_loss(x, yb, 32, "relu")
            loss.backward()
            torch.cuda.synchronize()
            out[side] = (loss.detach().clone(),
                         {n: p.grad.detach().clone() for n, p in mod.named_parameters() if p.requires_grad})
    finally:
        LY.DYN_WGRAD_SIDE = True
    assert torch.equal(out[True][0], out[False][0])
    for n, a in out[True][1].items():
        b = out[False][1][n]
        if "dyn_fun" in n:
            assert torch.equal(a, b), n
        else:
            torch.testing.assert_close(a, b, rtol=2e-4, atol=1e-7, msg=n)


def test_split_backward_entry_points_equal_one_call():
    """fiode_odetrain_backward_x (adjoint sweep + dL/dx_feat in k_ot_gx) followed by
    fiode_odetrain_backward_weights = the one-call fiode_odetrain_backward: the weight gradients bit
    for bit; dL/dx_feat is the same sum in another order (float32 rounding)."""
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(128, 0.1, False, 31)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    mk = torch.from_numpy(masks).to(dev)
    g = torch.Generator(device="cpu").manual_seed(2)
    gy = torch.randn(128, 10, generator=g).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=mk)
    one, _ = ops.odetrain_backward(gy, xt, w, dyn, cfg, ws)
    one = {k: v.clone() for k, v in one.items()}
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=mk)
    gx = ops.odetrain_backward_x(gy, xt, w, dyn, cfg, ws)
    wg = ops.odetrain_backward_weights(xt, w, dyn, cfg, ws)
    torch.cuda.synchronize()
    for k in KEYS:
        assert torch.equal(wg[k], one[k]), k
    torch.testing.assert_close(gx, one["x_feat"], rtol=1e-5, atol=1e-6 * float(one["x_feat"].abs().max()))


@pytest.mark.parametrize("B", [1, 128, 300])
def test_ode_nll_matches_torch(B):
    """ODENllFn (fiode_ode_nll) = F.nll_loss(torch.log(y_hat), y) (pl_modules.py:494-497), forward
    and backward, on simplex rows."""
    import torch.nn.functional as F
    from fiode_amd.lyapunov import ODENllFn
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(B)
    yh = torch.softmax(torch.randn(B, 10, generator=g), -1).to(dev)
    y = torch.randint(0, 10, (B,), generator=g).to(dev)
    a, b = yh.clone().requires_grad_(True), yh.clone().requires_grad_(True)
    la = ODENllFn.apply(a, y)
    lb = F.nll_loss(torch.log(b), y)
    (la * 0.37).backward()
    (lb * 0.37).backward()
    torch.cuda.synchronize()
    assert abs(float(la) - float(lb)) <= 1e-6 * max(1.0, abs(float(lb)))
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("p", [0.2, 0.98])
def test_ode_loss_mix_matches_torch(p):
    """ODELossMixFn (fiode_ode_loss_mix) = loss * (1 - p) + nll(log y_hat) * p (pl_modules.py:494-500),
    value and gradients w.r.t. loss and y_hat."""
    import torch.nn.functional as F
    from fiode_amd.lyapunov import ODELossMixFn
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(7)
    yh = torch.softmax(torch.randn(128, 10, generator=g), -1).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    l0 = torch.tensor(0.731, device=dev)
    a, la = yh.clone().requires_grad_(True), l0.clone().requires_grad_(True)
    b, lb = yh.clone().requires_grad_(True), l0.clone().requires_grad_(True)
    ta, ode_a = ODELossMixFn.apply(la, a, y, p)
    ode_b = F.nll_loss(torch.log(b), y)
    tb = lb * (1.0 - p) + ode_b * p
    (ta * 1.3).backward()
    (tb * 1.3).backward()
    torch.cuda.synchronize()
    assert abs(float(ta) - float(tb)) <= 2e-6 * max(1.0, abs(float(tb)))
    assert abs(float(ode_a) - float(ode_b)) <= 1e-6 * max(1.0, abs(float(ode_b)))
    torch.testing.assert_close(la.grad, lb.grad, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)


def test_philox_keep_rate_p05():
    """The train_ode solve's Philox dropout words keep half of the hidden units: over the 40
    evals x B rows x 2 layers, the fraction of kept units in the saved post-activation layout
    (a kept unit can still be 0 after the ReLU, so measured on pre-ReLU-independent data: the
    keep words themselves, read back through the saved a1 of a zero-bias, all-positive probe)."""
    from fiode_amd import _lib as L
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(128, 0.1, False, 11)
    w = {k: v.clone() for k, v in w.items()}
    # probe: layer-1 pre-activations all > 0 (u = b1 + bx large, Q1 = 0), so a1 = keep * 2 * z1
    w["Q1"].zero_(); w["Qx"].zero_(); w["b1"].fill_(1.0); w["bx"].fill_(1.0)
    c = ops.odetrain_config(128, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3, offset=7)
    y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, c)
    torch.cuda.synchronize()
    a1 = ops.odetrain_saved(ws, c)["a1"]                    # [B, E, M]
    rate = float((a1 > 0).float().mean())
    assert abs(rate - 0.5) < 3e-3, rate                     # 655k Bernoulli(1/2) draws: std 6e-4
    per_eval = (a1 > 0).float().mean(dim=(0, 2)).cpu()
    assert float((per_eval - 0.5).abs().max()) < 0.02


def test_exchange_timeout_poisons_output(monkeypatch):
    """A workgroup that never publishes its QP-exit mask (FIODE_DEBUG_DROP_PUBLISH test hook: as if
    it were not resident): the bounded spin ends, status 4 is recorded, y_hat is NaN for the tiles
    that used a partial AND, and the module's sticky status check raises."""
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(64, 0.25, True, 12)
    monkeypatch.setenv("FIODE_DEBUG_DROP_PUBLISH", "1")
    y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                     masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    assert int(st[3]) == 4
    assert torch.isnan(y).any()
    import bench
    mod = bench.build_module(dev, seed=0, train_ode=True)
    xb = torch.rand(32, 3, 32, 32, device=dev)
    yb = torch.randint(0, 10, (32,), device=dev)
    loss = mod.compute_loss(xb, yb, 32, "relu")
    torch.cuda.synchronize()
    assert mod.device_status() == 4 and torch.isnan(loss)
    with pytest.raises(RuntimeError, match="timed out"):
        mod.check_device_status()


def test_feature_reuse_equals_reference_order():
    """The train_ode branch reuses the step's backbone features (one backbone pass); the reference
    re-runs the backbone inside self.model(x) (pl_modules.py:491).  With both backbone passes on
    the same stream (no Cayley-map prefetch) they give bit-identical features, so the loss and
    every dynamics gradient are identical and the backbone gradients agree up to float32 summation
    order (the two branches' feature gradients meet before the backbone instead of inside it).

    (With the prefetch on, the first pass's Cayley maps come from side streams whose library GEMMs
    round differently: the features then differ by ~1e-6, and the QP backward's active set -- a
    sign test on rounding noise, DESIGN.md section 5 -- flips for a few rows, which moves the
    gradients by a few percent: a property of the reference's gradient, tools/probes/cse_probe.py.)"""
    import bench
    dev = _dev()
    x = torch.rand(32, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    yb = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(4))
    out = {}
    for reuse in (True, False):
        mod = bench.build_module(dev, seed=0, train_ode=True)
        mod.parallel_cayley = False
        with torch.no_grad():          # the first forward initialises the conv alphas (a different path)
            mod.init_coordinates(x, mod.dyn_fun)
        mod.ode_reuse_features = reuse
        mod._rng_offset = 0
        feats = []
        hook = mod.init_coordinates.param_map.register_forward_hook(lambda m, i, o: feats.append(o.detach().clone()))
        loss = mod.compute_loss(x, yb, 32, "relu")
        hook.remove()
        loss.backward()
        torch.cuda.synchronize()
        assert len(feats) == (1 if reuse else 2)
        if not reuse:
            assert torch.equal(feats[0], feats[1])
        out[reuse] = (loss.detach().clone(), {n: p.grad.detach().clone() for n, p in mod.named_parameters()
                                              if p.requires_grad})
    (la, ga), (lb, gb) = out[True], out[False]
    assert torch.equal(la, lb)
    errs = {}
    for n in ga:
        if n.startswith("model.dyn_fun."):
            assert torch.equal(ga[n], gb[n]), n
        else:
            scale = float(gb[n].abs().max()) + 1e-12
            errs[n] = float((ga[n] - gb[n]).abs().max()) / scale
    print("backbone gradient max relative differences:", sorted(errs.items(), key=lambda kv: -kv[1])[:4])
    # a CayleyLinear's alpha gradient is one scalar, <dL/dX, W> / ||W|| over all cout x cin
    # entries with terms of both signs: its relative rounding spread is a few times a tensor's
    for n, e in errs.items():
        assert e <= (3e-4 if n.endswith(".alpha") else 1e-4), (n, e)


@pytest.mark.parametrize("scale_nominal,mode", [(False, "philox"), (True, "given")])
def test_forward_qp_bit_exact_per_eval(scale_nominal, mode):
    """Every eval's QP in the train_ode forward (three bisection iterations per round over the row's
    lanes, speculation to the previous exit + 3, the cross-tile exit exchange) equals the sequential
    reference bisection with the batch-global exit (barrier_projection.py:232-255) on the device's
    own (lower, nominal), bit for bit: mu, v and therefore the exit iteration of all 40 evals."""
    from fiode_amd import _lib as L
    ops, dev, P, x, h0, labels, cfg, E, masks, w, dyn = _case(128, 0.1, scale_nominal, 21)
    if mode == "philox":
        cfg = ops.odetrain_config(128, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=4, offset=2)
        y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg)
    else:
        y, st, ws = ops.odetrain_forward(torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev), w, dyn, cfg,
                                         masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    sv = {k: v.cpu().numpy() for k, v in ops.odetrain_saved(ws, cfg).items()}
    for e in range(E):
        q = O.qp_forward(sv["lower"][:, e], sv["nominal"][:, e], 30, 1e-4)
        assert np.array_equal(sv["mu"][:, e], q.mu), e
        assert np.array_equal(sv["v"][:, e], q.v), e
    assert int(st[2]) == q.iters
