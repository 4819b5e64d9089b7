"""Shared helpers for the test-suite (deterministic synthetic inputs)."""
import numpy as np

from oracle import fiode_oracle as O


def make_params(seed=0, C=10, M=128, X=10, bias_scale=0.1):
    rng = np.random.default_rng(seed)
    def lin(o, i):
        s = 1.0 / np.sqrt(i)
        W = rng.uniform(-s, s, (o, i))
        return O.cayley_linear_weight(W, np.linalg.norm(W))
    P = O.DynParams(
        Q1=lin(M, C), b1=rng.uniform(-bias_scale, bias_scale, M),
        Qx=lin(M, X), bx=rng.uniform(-bias_scale, bias_scale, M),
        Q2=lin(M, M), b2=rng.uniform(-bias_scale, bias_scale, M),
        Q3=lin(C, M), b3=rng.uniform(-bias_scale, bias_scale, C))
    return P.astype32()


def make_step_inputs(B=4, S=8, C=10, M=128, X=10, seed=1, S1=None, dropout=True, kappa=2.0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, C, B)
    S1 = S - max(1, S // 5) if S1 is None else S1
    ud = rng.exponential(1.0, (S1, C)).astype(np.float32)
    cd = rng.exponential(1.0, (B, S - S1, C)).astype(np.float32)
    h = O.composite_h(y, ud, cd)
    x = rng.normal(0, 1, (B, X)).astype(np.float32)
    N = B * S
    if dropout:
        m = [rng.integers(0, 2, (N, M)).astype(np.uint8) for _ in range(4)]
    else:
        m = [None] * 4
    return O.StepInputs(x_feat=x, y=y, h=h, S=S, mask1=m[0], mask2=m[1], lmask1=m[2], lmask2=m[3],
                        kappa=kappa)
