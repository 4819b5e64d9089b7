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


def _attempt_log(ws, cfg, A):
    """(accept decisions, dt, error ratio) per attempt from the device's saved attempt log."""
    at = __import__("fiode_amd.ops", fromlist=["odetrain_saved"]).odetrain_saved(ws, cfg)["attempts"][:A].cpu()
    return [bool(a) for a in at[:, 3].numpy()], at[:, 1].numpy(), at[:, 2].numpy()


@pytest.mark.parametrize("B,seed", [(128, 4), (1024, 8)])
def test_controller_unpinned_matches_float64_oracle(B, seed):
    """The train-mode dopri5 solve against the float64 restatement (oracle/dopri5_train.py) with
    NOTHING pinned but the dropout masks: the oracle runs its own QPs (own batch-global exits) and
    its own step-size controller, so torchdiffeq's accept rule ratio <= 1 (models.py:235-241,
    RKAdaptiveStepsizeODESolver) decides every attempt on the oracle side.  B = 1,024 is configs[4]'s
    per-rank batch.  The device must take the same attempts (NFE, accept / reject sequence), its
    per-attempt dt and error ratio must agree to float32-vs-float64 precision, and y(t1) must agree
    within 1e-4: each eval's QP solution is only fixed to the bisection resolution (the batch-global
    exit at max |eps| < 1e-4), and the solve chains ~100-200 evals through the stages (measured: 7e-6
    at B = 128, 1.1e-5 at B = 1,024; profiles/r05a/oracle_pinning.log)."""
    ops, dev, P, x, h0, cfg, masks, w = _setup(B, seed, 1e-3)
    dyn = ops.DynCfg(scale_nominal=False, dropout=0.5)
    xt, h0t = torch.from_numpy(x).to(dev), torch.from_numpy(h0).to(dev)
    y, st, ws = ops.odetrain_forward(xt, h0t, w, dyn, cfg, masks=torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0, s
    nfe, A = int(s[0]), int(s[6])
    acc, dts, ratios = _attempt_log(ws, cfg, A)
    W64 = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).double() for k in KEYS}
    tr = D.Trace()
    with torch.no_grad():
        yr, info = D.dopri5_train(torch.from_numpy(x).double(), torch.from_numpy(h0).double(), W64,
                                  torch.from_numpy(masks), 0.0, 1.0, 1e-3, 1e-3, scale_nominal=False, p=0.5,
                                  max_attempts=64, trace=tr)
    oacc = [r["accept"] for r in tr.attempts]
    odt = np.array([float(r["dt"]) for r in tr.attempts])
    orat = np.array([float(r["ratio"]) for r in tr.attempts])
    print(f"B={B}: device nfe {nfe} attempts {A} ({sum(acc)} accepted); oracle nfe {info['nfe']} attempts "
          f"{len(oacc)} ({sum(oacc)} accepted); min |ratio - 1| {float(np.abs(orat - 1).min()):.3e}")
    assert (info["nfe"], oacc) == (nfe, acc)
    assert np.allclose(dts, odt, rtol=1e-3, atol=0), np.abs(dts / odt - 1).max()
    assert np.allclose(ratios, orat, rtol=2e-2, atol=1e-3), np.abs(ratios - orat).max()
    err = float((y.cpu().double() - yr).abs().max())
    print(f"B={B}: max |y_dev - y_oracle| {err:.3e}")
    assert err <= 1e-4, err


@pytest.mark.parametrize("B,S", [(1024, 1024), (128, 256)])
def test_nan_state_reproduced_by_oracle(B, S):
    """configs[4] (B = 1,024 x S = 1,024) and configs[2] (B = 128 x S = 256), train_ode dopri5 tol
    1e-3: the captured training step of bench.py's module skips a step on a NaN loss -- F.nll_loss(torch.log(y_hat), y)
    (pl_modules.py:494-497) of a solve whose y_hat[label] <= 0 for some images.  At that state (the
    parameters after two updates, the same batch), the solve is re-run on the device with the same
    Philox dropout stream and its keep words exported, and the float64 oracle (own QPs, own
    controller, the same keep masks) is run on the same features and weights: the oracle must also
    drive those images' label component to <= 0, i.e. the reference's own arithmetic takes the log of
    a non-positive value there and the NaN is not a device artefact.  A float32 run of the oracle is
    reported beside it."""
    import bench
    from fiode_amd import _lib as L, ops
    from fiode_amd.graph_step import GraphTrainStep
    from tests.test_gpu_sampler import masks_from_keep_words
    dev = _dev()
    # configs[4]'s NaN steps come at the third replay; configs[2]'s are rarer (3 of 25 bench replays
    # in round 4) and move with the last bits of the backbone's arithmetic, so at B = 128 several
    # synthetic batches are searched (the first NaN replay found is the state checked)
    batch_seeds, reps = ([1234], 30) if B == 1024 else ([1234, 1, 2, 3, 4, 5, 6, 7], 60)
    nan_step = None
    for bseed in batch_seeds:
        mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5", h_sample=S)
        mod.seed = 1000
        opt = mod.configure_optimizers(capturable=True)[0][0]
        g = torch.Generator(device="cpu").manual_seed(bseed)
        x = torch.rand(B, 3, 32, 32, generator=g).to(dev)
        y = torch.randint(0, 10, (B,), generator=g).to(dev)
        gs = GraphTrainStep(mod, opt, x, y, check_every=0)
        for i in range(reps):
            loss = gs.step()
            torch.cuda.synchronize()
            if not bool(torch.isfinite(loss).all()):
                nan_step = i
                break
        if nan_step is not None:
            break
        gs.close()
    if nan_step is None and B == 128:
        pytest.skip(f"no NaN step in {reps} replays of {len(batch_seeds)} batches at B = 128 with this build's rounding")
    assert nan_step is not None, f"no NaN step in {reps} replays"
    print(f"batch seed {bseed}")
    assert gs.skipped_steps() == 1                 # the guard kept the update away
    yh_graph = mod.last_plan["y_hat"].detach().clone()
    counter = int(mod.rng_counter.item()) - 1      # the replay's Philox offset (advanced after it)
    gs.close()
    with torch.no_grad():
        feat = mod.init_coordinates.param_map(x).float().contiguous()
        w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.0, L.FIODE_DROPOUT_PHILOX, seed=mod.seed, offset=0, method="dopri5",
                              rtol=1e-3, atol=1e-3, max_attempts=64)
    h0 = torch.full((B, 10), 0.1, device=dev)
    yd, st, ws = ops.odetrain_forward(feat, h0, w, ops.DynCfg(scale_nominal=False, dropout=0.5), cfg,
                                      offset_dev=torch.tensor([counter], dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[3] == 0, s
    nfe, A = int(s[0]), int(s[6])
    lab = y.long().cpu()
    yl_dev = yd.cpu().double().gather(1, lab[:, None])[:, 0]
    yl_graph = yh_graph.cpu().double().gather(1, lab[:, None])[:, 0]
    neg = torch.nonzero(yl_dev <= 0)[:, 0]
    print(f"NaN at replay {nan_step}; graph y_hat[label] <= 0: {int((yl_graph <= 0).sum())} "
          f"(min {float(yl_graph.min()):.3e}); re-run: {len(neg)} (min {float(yl_dev.min()):.3e}), nfe {nfe}")
    assert len(neg) >= 1
    masks = masks_from_keep_words(ops.odetrain_saved(ws, cfg)["keep_words"][:nfe].reshape(nfe * 2, B, 4)) \
        .reshape(nfe, 2, B, 128).cpu()
    acc, _, _ = _attempt_log(ws, cfg, A)
    res = {}
    for dt_ in (torch.float64, torch.float32):
        Wo = {k: v.cpu().to(dt_) for k, v in w.items()}
        tr = D.Trace()
        with torch.no_grad():
            yr, info = D.dopri5_train(feat.cpu().to(dt_), h0.cpu().to(dt_), Wo, masks, 0.0, 1.0, 1e-3, 1e-3,
                                      scale_nominal=False, p=0.5, max_attempts=64, trace=tr)
        yl = yr.double().gather(1, lab[:, None])[:, 0]
        res[dt_] = (yl, info["nfe"], [r["accept"] for r in tr.attempts])
        print(f"oracle {dt_}: nfe {info['nfe']} (device {nfe}), accepts equal {res[dt_][2] == acc}, "
              f"y_hat[label] <= 0: {int((yl <= 0).sum())} (min {float(yl.min()):.3e}); at the device's "
              f"negative images: {[round(float(v), 5) for v in yl[neg]]} vs device "
              f"{[round(float(v), 5) for v in yl_dev[neg]]}")
    yl64 = res[torch.float64][0]
    # the reference's arithmetic (float64 restatement, its own QPs and controller) also reaches a
    # non-positive label component: log(y_hat) is NaN there too
    assert bool((yl64 <= 0).any())
    assert bool((yl64[neg] <= 0).any())
    # and it reaches the device's values at those images (the same solve within float32 rounding)
    assert float((yl64[neg] - yl_dev[neg]).abs().max()) <= 1e-4
