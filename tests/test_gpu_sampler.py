"""GPU parity of the in-kernel sampler fan-out and of the production (Philox) mode of
fiode_lyap_step, through the C-ABI.

* Given Exp(1) draws (fiode_lyap_io.exp_draws), the device samplers must reproduce the oracle's
  restatement of UniformSimplexSampling / CorrectConeSampling / DecisionBoundarySampling
  (sampling/sampler.py:34-38, 113-128, 139-153) BIT FOR BIT, labels 0 and 9 and ties included.
* In Philox mode (what bench.py times) the exported Exp(1) variates fed to the oracle give the
  exported samples bit for bit, and the whole step equals the GIVEN-mode step fed the exported
  samples and dropout keep words bit for bit (scalars, V, V-dot, f, grads).
* Dropout keep rates: p = 0.5 (one Philox bit per unit) and a general p (byte threshold).
"""
import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from tests._util import make_params

pytestmark = pytest.mark.gpu
C, M = 10, 128


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


def masks_from_keep_words(kw: torch.Tensor) -> torch.Tensor:
    """[4, N, 4] int32 keep words (bit t of word mb = hidden 32 mb + t) -> uint8 [4, N, 128]."""
    w = kw.to(torch.int64) & 0xFFFFFFFF
    bits = (w[..., None] >> torch.arange(32, device=kw.device)) & 1
    return bits.reshape(kw.shape[0], kw.shape[1], 4 * 32).to(torch.uint8)


def _labels(B, rng):
    y = rng.integers(0, C, B)
    y[0], y[1] = 0, C - 1          # the first and the last class always present
    return y


def _step(dev, y, S, S1, sampler, draws=None, dropout_mode=None, masks=None, h=None, seed=77, offset=5,
          scale_nominal=False, dropout=0.5, P=None):
    ops, L = _ops()
    P = P if P is not None else make_params(seed=3)
    B = len(y)
    x = torch.from_numpy(np.random.default_rng(4).normal(size=(B, 10)).astype(np.float32)).to(dev)
    mode = L.FIODE_DROPOUT_OFF if dropout_mode is None else dropout_mode
    sc, gr, dbg = ops.lyap_step(x, torch.from_numpy(np.asarray(y, np.int64)).to(dev), _wt(P, dev),
                                ops.DynCfg(scale_nominal=scale_nominal, dropout=dropout), sample_size=S, n_uniform=S1,
                                sampler=sampler, dropout_mode=mode, seed=seed, offset=offset,
                                exp_draws=None if draws is None else torch.from_numpy(draws).to(dev),
                                masks=masks, h=h, debug=True)
    torch.cuda.synchronize()
    return sc, gr, dbg


def _cone_ties(cd, y):
    """Craft ties into CorrectCone draws [B, S2, C]: two coordinates at the row max, an all-equal
    row, the label already the max, and the label tied with another coordinate at the max."""
    B = cd.shape[0]
    cd[:, 0, 2] = cd[:, 0, 7] = 9.0
    cd[:, 1, :] = 1.0
    for b in range(B):
        cd[b, 2, y[b]] = 9.0
        cd[b, 3, y[b]] = cd[b, 3, (y[b] + 1) % C] = 9.0
        cd[b, 4, (y[b] + 3) % C] = cd[b, 4, (y[b] + 5) % C] = 9.0
    return cd


def test_composite_sampler_given_draws_bit_exact():
    dev = _dev()
    _, L = _ops()
    rng = np.random.default_rng(0)
    B, S, S1 = 12, 40, 25
    y = _labels(B, rng)
    ud = rng.exponential(1.0, (S1, C)).astype(np.float32)
    ud[0, :] = 2.0                                         # an all-equal uniform draw
    cd = _cone_ties(rng.exponential(1.0, (B, S - S1, C)).astype(np.float32), y)
    draws = np.concatenate([ud.ravel(), cd.ravel()])
    _, _, dbg = _step(dev, y, S, S1, L.FIODE_SAMPLER_COMPOSITE, draws=draws)
    h = dbg["h"].cpu().numpy()
    ref = O.composite_h(y, ud, cd)
    assert np.array_equal(h, ref), float(np.abs(h - ref).max())
    assert np.array_equal(dbg["exp_draws"].cpu().numpy(), draws)
    hb = h.reshape(B, S, C)
    cone = hb[:, S1:]
    assert (cone[np.arange(B), :, y] == cone.max(-1)).all()   # CorrectCone: the label holds the max (ties kept)


def test_decision_boundary_sampler_given_draws_bit_exact():
    dev = _dev()
    _, L = _ops()
    rng = np.random.default_rng(1)
    B, S = 10, 17
    y = np.arange(B)                                       # every label 0..9
    z = rng.exponential(1.0, (B, S, C - 1)).astype(np.float32)
    z[:, 0, :] = 1.0                                       # all equal
    z[:, 1, 3] = z[:, 1, 5] = 7.0                          # tie at the max
    z[:, 2, 0] = z[:, 2, 8] = 7.0                          # tie at the ends
    _, _, dbg = _step(dev, y, S, S, L.FIODE_SAMPLER_DECISION_BOUNDARY, draws=z.ravel())
    h = dbg["h"].cpu().numpy()
    ref = O.decision_boundary_samples(z, y).reshape(B * S, C)
    assert np.array_equal(h, ref), float(np.abs(h - ref).max())
    hb = h.reshape(B, S, C)
    others = np.where(np.arange(C)[None, None, :] == y[:, None, None], -1.0, hb).max(-1)
    assert np.array_equal(hb[np.arange(B), :, y], others)   # h_y = max_{j != y} h_j by construction


def test_decision_boundary_step_equals_given_step():
    """The DECISION_BOUNDARY sampler through the whole fused step = the GIVEN step on the oracle's
    samples, bit for bit (certify YAML's sampler, configs/certify/cifar_certify.yaml:5-7)."""
    dev = _dev()
    _, L = _ops()
    rng = np.random.default_rng(2)
    B, S = 16, 32
    y = _labels(B, rng)
    z = rng.exponential(1.0, (B, S, C - 1)).astype(np.float32)
    h_ref = O.decision_boundary_samples(z, y).reshape(B * S, C)
    masks = torch.from_numpy(rng.integers(0, 2, (4, B * S, M)).astype(np.uint8)).to(dev)
    a = _step(dev, y, S, S, L.FIODE_SAMPLER_DECISION_BOUNDARY, draws=z.ravel(), dropout_mode=L.FIODE_DROPOUT_GIVEN,
              masks=masks, scale_nominal=True)
    b = _step(dev, y, S, S, L.FIODE_SAMPLER_GIVEN, h=torch.from_numpy(h_ref).to(dev),
              dropout_mode=L.FIODE_DROPOUT_GIVEN, masks=masks, scale_nominal=True)
    _assert_steps_equal(a, b)


def _assert_steps_equal(a, b):
    sa, ga, da = a
    sb, gb, db = b
    assert torch.equal(sa, sb), (sa.cpu().numpy(), sb.cpu().numpy())
    for k in ("h", "V", "Vdot", "f", "f_log", "qp_lower", "qp_nominal", "g_ftilde"):
        assert torch.equal(da[k], db[k]), k
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k


@pytest.mark.parametrize("sampler_name", ["COMPOSITE", "DECISION_BOUNDARY"])
def test_philox_sampler_equals_oracle_on_its_draws(sampler_name):
    dev = _dev()
    _, L = _ops()
    sampler = getattr(L, f"FIODE_SAMPLER_{sampler_name}")
    rng = np.random.default_rng(3)
    B, S, S1 = 64, 256, 204
    y = _labels(B, rng)
    _, _, dbg = _step(dev, y, S, S1 if sampler_name == "COMPOSITE" else S, sampler, seed=1234, offset=9)
    e = dbg["exp_draws"].cpu().numpy()
    h = dbg["h"].cpu().numpy()
    if sampler_name == "COMPOSITE":
        ud = e[:S1 * C].reshape(S1, C)
        cd = e[S1 * C:].reshape(B, S - S1, C)
        ref = O.composite_h(y, ud, cd)
    else:
        ref = O.decision_boundary_samples(e.reshape(B, S, C - 1), y).reshape(B * S, C)
    assert np.array_equal(h, ref), float(np.abs(h - ref).max())
    # the Philox variates are Exp(1): mean 1, P(e > ln 2) = 1/2, no zeros / infinities
    assert np.isfinite(e).all() and (e >= 0).all()
    assert abs(e.mean() - 1.0) < 0.01, e.mean()
    assert abs((e > np.log(2.0)).mean() - 0.5) < 0.01


@pytest.mark.parametrize("scale_nominal", [True, False])
def test_philox_step_equals_given_step_bit_exact(scale_nominal):
    """The benched production mode (Philox samples + Philox dropout words) = the GIVEN-mode step
    fed its exported samples and keep masks, bit for bit."""
    dev = _dev()
    _, L = _ops()
    rng = np.random.default_rng(4)
    B, S, S1 = 32, 64, 51
    y = _labels(B, rng)
    a = _step(dev, y, S, S1, L.FIODE_SAMPLER_COMPOSITE, dropout_mode=L.FIODE_DROPOUT_PHILOX, seed=99, offset=17,
              scale_nominal=scale_nominal)
    masks = masks_from_keep_words(a[2]["keep_words"])
    b = _step(dev, y, S, S1, L.FIODE_SAMPLER_GIVEN, h=a[2]["h"].clone(), dropout_mode=L.FIODE_DROPOUT_GIVEN,
              masks=masks, scale_nominal=scale_nominal)
    _assert_steps_equal(a, b)
    # and GIVEN mode echoes the masks it was fed as keep words
    assert torch.equal(b[2]["keep_words"], a[2]["keep_words"])


@pytest.mark.parametrize("p", [0.5, 0.3])
def test_philox_dropout_keep_rate(p):
    dev = _dev()
    _, L = _ops()
    rng = np.random.default_rng(5)
    B, S = 64, 256
    y = _labels(B, rng)
    _, _, dbg = _step(dev, y, S, 204, L.FIODE_SAMPLER_COMPOSITE, dropout_mode=L.FIODE_DROPOUT_PHILOX, seed=5,
                      offset=3, dropout=p)
    m = masks_from_keep_words(dbg["keep_words"]).float()          # [4, N, 128]
    expect = 0.5 if p == 0.5 else round((1.0 - p) * 256) / 256.0  # byte threshold for general p
    rates = m.mean(dim=(1, 2)).cpu().numpy()
    # 4.2M Bernoulli draws per set: std ~2.4e-4
    assert np.abs(rates - expect).max() < 2e-3, (rates, expect)
    per_unit = m.mean(dim=1).cpu().numpy()                        # [4, 128]: no stuck hidden unit
    assert np.abs(per_unit - expect).max() < 0.03
    # the 4 mask sets (loss L1/L2, logging L1/L2) are different draws
    for i in range(4):
        for j in range(i + 1, 4):
            agree = (m[i] == m[j]).float().mean().item()
            assert abs(agree - (expect ** 2 + (1 - expect) ** 2)) < 3e-3, (i, j, agree)
