"""BASELINE configs at their full sizes on the MI355X (configs[3], configs[4]), checked against the
oracle where the oracle finishes in seconds and by size-independent properties elsewhere.

* configs[3] -- certification on the T=40 grid (certify_lipschitz.py:100-143): one image over all
  G = 41,320,837 grid rows of its label, in cfg.batches = 10 slices of 4,132,083 rows plus the
  7-row tail slice (G % 10 = 7).  The tail slice (its own batch-global QP exit) is recomputed by
  the oracle from the unranked grid rows; every slice is finite and violation_larger_T <
  violation (the Lipschitz slack is positive).
* configs[4] -- the fused training step at B=1024 x S=1024 (N = 1,048,576 rows per rank):
  Philox samples, injected dropout masks.  With the QP inputs pinned to the device's (see
  tests/test_gpu_lyap.py) the oracle reproduces the exit iterations, V / V-dot, the loss (1e-5
  relative) and the effective batch size exactly; the MLP outputs of 4,096 sampled rows match the
  oracle's MLP within 2e-5.
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


def test_config4_certify_full_T40_grid():
    from fiode_amd import ops
    dev = _dev()
    T, label, batches = 40, 7, 10
    P = make_params(seed=44)
    x = np.random.default_rng(4).normal(size=10).astype(np.float32)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    grid = ops.certify_grid(T, device=dev)
    G = grid.shape[0]
    assert G == 41_320_837
    out, it = ops.certify_image(torch.from_numpy(x).to(dev), label, grid, w,
                                ops.DynCfg(scale_nominal=False, dropout=0.0), T=T, batches=batches)
    torch.cuda.synchronize()
    o, its = out.cpu().numpy(), it.cpu().numpy()
    slices = O.certify_batches(G, batches)
    assert len(slices) == 11 and slices[-1] == (10 * 4_132_083, G) and G - slices[-1][0] == 7
    assert o.shape == (11, 2) and np.isfinite(o).all()
    assert (o[:, 1] < o[:, 0]).all()
    assert ((its >= 0) & (its <= 29)).all()
    # the 7-row tail slice, recomputed by the oracle from the unranked rows (its own QP exit)
    f = O.db_count_table(10, T)
    tail = np.array([O.db_unrank(r, 10, T, f) for r in range(slices[-1][0], G)], np.int64)
    assert np.array_equal(grid[slices[-1][0]:].cpu().numpy().astype(np.int64), tail)
    vmax, vtmax = O.certify_image(x, label, tail, P, O.DynConfig(scale_nominal=False),
                                  O.CertifyConst(T=T, batches=1))
    assert abs(o[-1, 0] - vmax[0]) <= 2e-3 and abs(o[-1, 1] - vtmax[0]) <= 2e-3, (o[-1], vmax, vtmax)


def test_config5_fused_step_B1024_S1024():
    from fiode_amd import ops, _lib as L
    dev = _dev()
    B, S = 1024, 1024
    S1 = O.split_samples(S, O.cifar_train_mixer(20))[0]          # epoch 20: (819, 205)
    N = B * S
    P = make_params(seed=55)
    rng = np.random.default_rng(55)
    x = rng.normal(size=(B, 10)).astype(np.float32)
    y = rng.integers(0, 10, B)
    y[0], y[1] = 0, 9
    g = torch.Generator(device=dev).manual_seed(5)
    masks = torch.randint(0, 2, (4, N, 128), dtype=torch.uint8, device=dev, generator=g)
    cfg = O.DynConfig(scale_nominal=False)
    w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
    sc, grads, dbg = ops.lyap_step(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), w,
                                   ops.DynCfg(scale_nominal=False, dropout=0.5), sample_size=S, n_uniform=S1,
                                   sampler=L.FIODE_SAMPLER_COMPOSITE, dropout_mode=L.FIODE_DROPOUT_GIVEN,
                                   kappa=2.0, seed=21, offset=3, masks=masks, debug=True)
    torch.cuda.synchronize()
    s = sc.cpu().numpy()
    for v in grads.values():
        assert torch.isfinite(v).all()
    h = dbg["h"].cpu().numpy()
    lower = dbg["qp_lower"].cpu().numpy()
    nom = dbg["qp_nominal"].cpu().numpy()
    y_rows = np.repeat(y.astype(np.int64), S)
    # loss pass with the QP inputs pinned: exit iteration, V, V-dot, loss, effective batch size
    q = O.qp_forward(lower, nom[0], cfg.qp_max_iter, cfg.qp_tol)
    assert int(s[3]) == q.iters
    V, js = O.decision_boundary_V(h, y_rows)
    Vd = O.vdot(q.v, y_rows, js)
    assert np.array_equal(dbg["V"].cpu().numpy(), V)
    assert np.array_equal(dbg["Vdot"].cpu().numpy(), Vd)
    viol = np.maximum((Vd + (np.float32(2.0) * V).astype(np.float32)).astype(np.float32), np.float32(0))
    loss = float(np.sum(viol, dtype=np.float64) / N)
    assert abs(s[0] - loss) <= 1e-5 * max(1.0, abs(loss)), (s[0], loss)
    assert int(s[1]) == int((viol > 0).sum())
    ql = O.qp_forward(lower, nom[1], cfg.qp_max_iter, cfg.qp_tol)
    assert int(s[4]) == ql.iters
    # the MLP at this size: 4,096 sampled rows against the oracle's
    rows = np.sort(rng.choice(N, 4096, replace=False))
    m = masks[:, torch.from_numpy(rows).to(dev)].cpu().numpy()
    u_rows = O.static_projection(x, P)[rows // S]
    ref = O.eval_dot(h[rows], u_rows, P, cfg, m[0], m[1], 0.5)
    scale = max(1.0, float(np.abs(ref.nominal).max()))
    err = float(np.abs(nom[0][rows] - ref.nominal).max())
    assert err <= 2e-5 * scale, err
