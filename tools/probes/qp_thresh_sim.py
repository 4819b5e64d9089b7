"""CPU simulation (not a test) of the threshold form of the QP bisection (barrier_projection.py:241-255)
on the QP inputs of a train_ode solve: checks that the certified-threshold decisions equal the
float32 bisection's own decisions bit for bit, and counts how many iterations of each 16-row wave
would still need the direct eps evaluation (the fallback).

Measured outcome (round 3): a HIP implementation of this scheme in k_ot_fwd
(Newton root + six certified points per row and eval, comparisons per iteration, frozen lanes
finished in the exit exchange's shadow) was bit-identical to the sequential bisection on every
seeded solve and on adversarial rows, but SLOWER: k_ot_fwd 263 -> 359 us (bisection phase 1.97 ->
3.24 us per eval).  At one wave per SIMD the per-row setup (3 Newton steps, 6 certificate
evaluations) costs more dependent VALU time than the ~17 sequential iterations it replaces, and
the late iterations (rows converged, bracket inside the rounding band of the root) still need the
direct evaluation.  Not kept.

python tools/probes/qp_thresh_sim.py [newton_iters] [delta_ulps]
"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
from oracle import fiode_oracle as O  # noqa: E402
from tests._util import make_params  # noqa: E402

F32 = np.float32
R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
DU = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
TOL = F32(1e-4)
START = sys.argv[3] if len(sys.argv) > 3 else "lo"
MAXIT = 30


def eps_fl(n, l, mu):
    d = (n - mu[:, None]).astype(F32)
    return O.row_sum_seq(np.maximum(d, l))


def thresholds(n, l):
    b = (n - l).astype(F32)
    lo0 = n.min(1)
    mu = lo0.copy() if START == "lo" else (n.sum(1, dtype=F32) / F32(10)).astype(F32)
    sl = l.sum(1, dtype=F32)
    for _ in range(R):
        t = (b - mu[:, None]).astype(F32)
        k = (t > 0).sum(1).astype(F32)
        e = (sl + np.maximum(t, 0).sum(1, dtype=F32)).astype(F32)
        mu = np.where(k > 0, (mu + e / np.maximum(k, 1)).astype(F32), mu)
    t = (b - mu[:, None]).astype(F32)
    k = np.maximum((t > 0).sum(1), 1).astype(F32)
    mag = (np.abs((n - mu[:, None]).astype(F32)) + np.abs(l)).sum(1).astype(F32)
    dl = (F32(DU) * F32(2.0 ** -24) * mag).astype(F32)
    tol = TOL
    pts = {"A": mu - (tol + dl) / k, "B": mu - (tol - dl) / k, "C": mu - dl / k,
           "D": mu + dl / k, "E": mu + (tol - dl) / k, "F": mu + (tol + dl) / k}
    pts = {kk: v.astype(F32) for kk, v in pts.items()}
    ev = {kk: eps_fl(n, l, v) for kk, v in pts.items()}
    inf = F32(np.inf)
    th = {"A": np.where(ev["A"] >= tol, pts["A"], -inf), "B": np.where(ev["B"] < tol, pts["B"], inf),
          "C": np.where(ev["C"] > 0, pts["C"], -inf), "D": np.where(ev["D"] < 0, pts["D"], inf),
          "E": np.where(ev["E"] > -tol, pts["E"], -inf), "F": np.where(ev["F"] <= -tol, pts["F"], inf)}
    return th, mu


def run(n, l, rows_per_wave=16):
    N = n.shape[0]
    th, mustar = thresholds(n, l)
    hi = (n - l).astype(F32).max(1)
    lo = n.min(1)
    unc = []
    conv_all = []
    for it in range(MAXIT):
        mu = ((hi - lo).astype(F32) * F32(0.5) + lo).astype(F32)
        e = eps_fl(n, l, mu)
        P, Nn, Cv = e > 0, e < 0, np.abs(e) < TOL
        p_s = mu <= th["C"]
        n_s = mu >= th["D"]
        cf_s = (mu <= th["A"]) | (mu >= th["F"])
        ct_s = (mu >= th["B"]) & (mu <= th["E"])
        sure = (p_s | n_s) & (cf_s | ct_s)
        # certified decisions must equal the direct ones
        assert np.all(~(sure & p_s) | (P & ~Nn)), it
        assert np.all(~(sure & n_s) | (Nn & ~P)), it
        assert np.all(~(sure & cf_s) | ~Cv), it
        assert np.all(~(sure & ct_s) | Cv), it
        unc.append(int((~sure).reshape(-1, rows_per_wave).any(1).sum()))
        conv_all.append(bool(Cv.all()))
        lo = np.where(P, mu, lo).astype(F32)
        hi = np.where(Nn, mu, hi).astype(F32)
    K = conv_all.index(True) if True in conv_all else MAXIT - 1
    return sum(unc[:K + 2]), unc[:K + 2], K


def main():
    B = 128
    P = make_params(seed=3)
    rng = np.random.default_rng(5)
    x = rng.normal(size=(B, 10)).astype(F32)
    h0 = np.full((B, 10), 0.1, F32)
    E = 40
    masks = (rng.random((E, 2, B, 128)) >= 0.5).astype(np.uint8)
    cfg = O.DynConfig(scale_nominal=False)
    _, recs = O.rk4_train(x, h0, P, cfg, 0.0, 1.0, 0.1, masks, 0.5)
    tot_w = tot_it = 0
    ks = []
    per_it = np.zeros(MAXIT)
    for e, (h, r) in enumerate(recs):
        uw, ur, K = run(r.nominal.astype(F32), r.lower.astype(F32))
        # iterations the kernel runs: to the exit K (+1 speculation margin)
        tot_w += uw
        per_it[:len(ur)] += ur
        tot_it += (K + 2) * (B // 16)
        ks.append(K)
    print("per-iteration uncertain waves (sum over evals):", per_it[:20].astype(int).tolist())
    print(f"R={R} delta={DU}ulp: uncertain wave-iterations {tot_w} of {tot_it} (to K+1); "
          f"exits K: min {min(ks)} max {max(ks)} mean {np.mean(ks):.1f}")


if __name__ == "__main__":
    main()
