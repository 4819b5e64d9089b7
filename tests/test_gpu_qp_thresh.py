"""The certified-threshold bisection of the persistent solves (tile16.h: qp_thresholds /
qp_bisect_thr / qp_bisect_frozen, used by k_ot_fwd) against the plain sequential bisection of
FastBarrierProjectionNoUpper (barrier_projection.py:241-255), through fiode_qp_bisect_trace: every
midpoint of every iteration bit for bit, and each 64-row group's convergence mask (the AND of the
rows' |eps| < tol bits) -- on QP inputs of a train_ode solve, random rows at several scales, and
adversarial rows (ties, all-inactive, all-equal, zeros, huge spreads, NaN / inf entries).

The reference here is numpy in float32 with the device's operation order: midpoint
(hi - lo) / 2 + lo, eps = sum_j max(nom_j - mu, lower_j) left to right, max / min as IEEE maxNum /
minNum (np.fmax / np.fmin: the device's v_max_f32 returns the non-NaN operand)."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import fiode_oracle as O
from tests._util import make_params

pytestmark = pytest.mark.gpu
F32 = np.float32
TOL = 1e-4


def _trace_ref(lower, nom, iters, tol=TOL):
    lower, nom = lower.astype(F32), nom.astype(F32)
    hi = np.fmax.reduce((nom - lower).astype(F32), axis=1)
    lo = np.fmin.reduce(nom, axis=1)
    n = nom.shape[0]
    mus = np.zeros((n, iters), F32)
    conv = np.zeros((n, iters), bool)
    for it in range(iters):
        mu = ((hi - lo).astype(F32) / F32(2) + lo).astype(F32)
        v = np.fmax((nom - mu[:, None]).astype(F32), lower)
        eps = v[:, 0].copy()
        for j in range(1, nom.shape[1]):
            eps = (eps + v[:, j]).astype(F32)
        mus[:, it] = mu
        conv[:, it] = np.abs(eps) < F32(tol)
        lo = np.where(eps > 0, mu, lo).astype(F32)
        hi = np.where(eps < 0, mu, hi).astype(F32)
    return mus, conv


def _run(lower, nom, iters=30):
    from fiode_amd import _lib as L
    dev = torch.device("cuda:0")
    n = nom.shape[0]
    lt = torch.from_numpy(np.ascontiguousarray(lower, F32)).to(dev)
    nt = torch.from_numpy(np.ascontiguousarray(nom, F32)).to(dev)
    mu = torch.empty((n, iters), dtype=torch.float32, device=dev)
    masks = torch.empty((n + 63) // 64, dtype=torch.int32, device=dev)
    L.check(L.lib().fiode_qp_bisect_trace(None, n, 10, lt.data_ptr(), nt.data_ptr(), iters, ct.c_float(TOL),
                                          mu.data_ptr(), masks.data_ptr()), "fiode_qp_bisect_trace")
    torch.cuda.synchronize()
    return mu.cpu().numpy(), masks.cpu().numpy().view(np.uint32)


def _check(lower, nom, iters=30):
    mu, masks = _run(lower, nom, iters)
    rmu, rconv = _trace_ref(lower, nom, iters)
    same = (mu.view(np.uint32) == rmu.view(np.uint32)) | (np.isnan(mu) & np.isnan(rmu))
    assert same.all(), np.argwhere(~same)[:5]
    n = nom.shape[0]
    for g in range((n + 63) // 64):
        rows = rconv[64 * g:64 * g + 64]
        want = 0
        for it in range(iters):
            if rows[:, it].all():
                want |= 1 << it
        assert int(masks[g]) == want, (g, hex(int(masks[g])), hex(want))


def _solve_inputs(B=128, step=0.25, seed=3, scale_nominal=False):
    P = make_params(seed=seed)
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(B, 10)).astype(F32)
    h0 = np.full((B, 10), 0.1, F32)
    E = 4 * int(round(1.0 / step))
    masks = (rng.random((E, 2, B, 128)) >= 0.5).astype(np.uint8)
    _, recs = O.rk4_train(x, h0, P, O.DynConfig(scale_nominal=scale_nominal), 0.0, 1.0, step, masks, 0.5)
    lower = np.concatenate([r.lower for _, r in recs]).astype(F32)
    nom = np.concatenate([r.nominal for _, r in recs]).astype(F32)
    return lower, nom


@pytest.mark.parametrize("scale_nominal", [False, True])
def test_threshold_bisection_on_solve_inputs(scale_nominal):
    lower, nom = _solve_inputs(scale_nominal=scale_nominal)
    _check(lower, nom)


@pytest.mark.parametrize("scale", [1e-3, 1.0, 20.0, 1e3])
def test_threshold_bisection_random_rows(scale):
    rng = np.random.default_rng(int(scale * 1000) % 9973)
    n = 64 * 37 + 5                                              # a ragged last group
    h = rng.dirichlet(np.ones(10), size=n).astype(F32)
    lower = (-100.0 * (np.exp(0.02 * h.astype(np.float64)) - 1.0)).astype(F32)
    nom = (rng.normal(size=(n, 10)) * scale).astype(F32)
    _check(lower, nom)


def test_threshold_bisection_adversarial_rows():
    rng = np.random.default_rng(11)
    rows_l, rows_n = [], []

    def add(l, nm):
        rows_l.append(np.asarray(l, F32))
        rows_n.append(np.asarray(nm, F32))
    z = np.zeros(10, F32)
    add(z, z)                                             # everything zero: eps = 0 at once
    add(z, np.full(10, 3.0))                              # all equal nominal
    add(np.full(10, -0.5), np.full(10, -0.5))             # nominal on the bounds (all inactive)
    add(-np.arange(10) * 0.1, np.arange(10) * 0.5)        # distinct breakpoints
    add(np.full(10, -1e-3), np.r_[1e4, np.zeros(9)])      # one huge coordinate
    add(np.full(10, -2.0), np.r_[np.full(5, 7.0), np.full(5, -7.0)])   # ties in pairs
    add(np.full(10, -1.0), np.r_[1e-20, np.zeros(9)])     # tiny spread
    add(z, np.r_[np.nan, np.ones(9)])                     # NaN nominal entry
    add(np.r_[np.nan, np.zeros(9)], np.ones(10))          # NaN bound
    add(z, np.r_[np.inf, np.ones(9)])                     # inf nominal entry
    add(np.full(10, -np.inf), np.ones(10))                # -inf bounds
    for _ in range(53):                                    # rows whose root sits on a breakpoint
        b = rng.normal(size=10).astype(F32)
        l = -np.abs(rng.normal(size=10)).astype(F32) * 0.1
        add(l, (b + l).astype(F32))
    lower, nom = np.stack(rows_l), np.stack(rows_n)
    _check(lower, nom)
    # each adversarial row alone (its own 64-row group: its own mask)
    for i in range(11):
        _check(lower[i:i + 1], nom[i:i + 1])
