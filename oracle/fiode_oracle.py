"""CPU oracle for the FI-ODE forward-invariance hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it; the product path (``fi-ode_amd``) never
does, and fails loudly when its HIP library is missing.

It restates, in numpy, the algorithm of the reference (yjhuangcd/FI-ODE, read as text under
/root/reference -- never imported) for the path named by
BASELINE.json ``north_star``:

  * sampler fan-out            sampling/sampler.py:24-38, 104-153, 169-216
  * mixer schedule             sampling/sampler_schedulers.py:14-77
  * Cayley-MLP dynamics        dynamics/classification.py:96-115
  * bisection QP fwd / bwd     barrier_projection/barrier_projection.py:217-313
  * DecisionBoundary V, jvp    lya_cands.py:79-94, pl_modules.py:403-412
  * hinge loss + logging pass  pl_modules.py:444-484
  * ODE solves (torchdiffeq 0.2.2 'rk4' = 3/8 rule, 'dopri5'), called at models.py:235-241

PARITY STATUS.  The reference cannot be imported or run in this environment (a denial recorded
in SURVEY.md section 8c binds every round), the reference ships no tests, fixtures or golden
vectors, torchdiffeq and the ortho_conv submodule are absent.  This oracle
is therefore pinned by (i) known-answer tests derived by hand from the reference source text,
(ii) an op-for-op torch-CPU restatement of the same source lines (``oracle/torch_ref.py``) whose
autograd/jvp semantics the closed-form backward here must reproduce, and (iii) analytic ODE
solutions.  Against the reference's own outputs it is **parity unpinned**.

Numerics conventions (the HIP kernels follow the same ones, which is what makes several
comparisons bit-exact):
  * state/activations are float32, as in the reference;
  * every reduction over the C=10 class axis is a sequential left-to-right float32 sum
    (the reference's ``torch.sum`` order is a vectorised cascade: differences are <= 1 ulp per
    add and only matter when a QP residual sits within 1 ulp of ``tol``);
  * ODE time arithmetic is float64, as torchdiffeq does.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

F32 = np.float32
C_DEFAULT = 10


# ---------------------------------------------------------------------------------------------
# sampler schedules -- sampling/sampler_schedulers.py
# ---------------------------------------------------------------------------------------------

def linear_scheduler_weight(epoch: int, rate: float, bias: float = 0.0, clamp: str = "min",
                            clamp_val: float = 0.0, start: int = 0) -> float:
    """``LinearScheduler.sampler_weight`` (sampler_schedulers.py:25-38)."""
    if epoch < start:
        return 0.0 if rate > 0 else 1.0
    w = (epoch - start) * rate + bias
    if clamp not in ("min", "max"):
        return w
    if clamp == "max":
        return min(w, clamp_val)
    return max(w, clamp_val)


def mixer_coefficients(unnormalised: Sequence[float], weights: Sequence[float]) -> np.ndarray:
    """``CompositeSamplerScheduler.get_mixer_coefficients`` (sampler_schedulers.py:72-77):
    float64 L1 normalisation with the reference's ``+ 1e-12``."""
    wc = np.asarray(unnormalised, dtype=np.float64) * np.asarray(weights, dtype=np.float64)
    return wc / (np.linalg.norm(wc, ord=1) + 1e-12)


def cifar_train_mixer(epoch: int) -> np.ndarray:
    """Mixer of configs/classification/cifar_train.yaml:17-28,43 (two LinearSchedulers)."""
    v1 = linear_scheduler_weight(epoch, rate=-0.02, bias=1.0, clamp="min", clamp_val=0.02, start=10)
    v2 = linear_scheduler_weight(epoch, rate=0.02, bias=0.0, clamp="max", clamp_val=0.98, start=10)
    return mixer_coefficients([v1, v2], [1.0, 1.0])


def split_samples(sample_size: int, coeffs: Sequence[float]) -> List[int]:
    """``CompositeSampler._coefficient_to_num_samples`` (sampler.py:181-192): floor split, the
    last sampler takes the remainder."""
    out: List[int] = []
    added = 0
    for c in coeffs:
        if len(out) == len(coeffs) - 1:
            out.append(sample_size - added)
            break
        s = math.floor(sample_size * float(c))
        added += s
        out.append(s)
    assert sum(out) == sample_size
    return out


# ---------------------------------------------------------------------------------------------
# samplers -- sampling/sampler.py.  Random draws are INPUTS (Exp(1) variates), so the oracle and
# the device kernels can be fed identical draws.
# ---------------------------------------------------------------------------------------------

def l1_normalize_rows(x: np.ndarray) -> np.ndarray:
    """``F.normalize(x, p=1, dim=-1)`` = x / max(sum|x|, 1e-12), sequential float32 sum."""
    x = np.asarray(x, dtype=F32)
    s = np.zeros(x.shape[:-1], dtype=F32)
    for j in range(x.shape[-1]):
        s = (s + np.abs(x[..., j])).astype(F32)
    s = np.maximum(s, F32(1e-12))
    return (x / s[..., None]).astype(F32)


def uniform_simplex(exp_draws: np.ndarray) -> np.ndarray:
    """``UniformSimplexSampling.forward`` (sampler.py:34-38): [S1,C] Exp(1) -> L1 normalised."""
    return l1_normalize_rows(exp_draws)


def correct_cone(exp_draws: np.ndarray, y: np.ndarray) -> np.ndarray:
    """``CorrectConeSampling.forward`` (sampler.py:113-128): [B,S2,C] Exp(1) -> L1 normalised,
    then the label coordinate and the row's (first-index) argmax coordinate swap values."""
    h = l1_normalize_rows(exp_draws).copy()
    B, S2, C = h.shape
    amax = np.argmax(h, axis=-1)                     # first index on ties (torch CPU max)
    hmax = np.take_along_axis(h, amax[..., None], -1)[..., 0]
    yy = np.broadcast_to(np.asarray(y)[:, None], (B, S2))
    hlab = np.take_along_axis(h, yy[..., None], -1)[..., 0]
    np.put_along_axis(h, yy[..., None], hmax[..., None], -1)
    np.put_along_axis(h, amax[..., None], hlab[..., None], -1)
    return h


def decision_boundary_samples(exp_draws: np.ndarray, y: np.ndarray) -> np.ndarray:
    """``DecisionBoundarySampling.forward`` (sampler.py:139-153): z in Exp(1)^(C-1) per row,
    raw = normalize([max z, z]); the label gets raw[0], the other classes get raw[1:] in order."""
    z = np.asarray(exp_draws, dtype=F32)
    B, S, Cm1 = z.shape
    raw = l1_normalize_rows(np.concatenate([z.max(-1, keepdims=True), z], -1))
    h = np.zeros((B, S, Cm1 + 1), dtype=F32)
    for b in range(B):
        yb = int(y[b])
        others = [c for c in range(Cm1 + 1) if c != yb]
        h[b, :, yb] = raw[b, :, 0]
        h[b, :, others] = raw[b, :, 1:].T
    return h


def composite_h(y: np.ndarray, uniform_draws: Optional[np.ndarray],
                cone_draws: Optional[np.ndarray]) -> np.ndarray:
    """``CompositeSampler.forward`` (sampler.py:195-216) for the training mix
    (Uniform [S1,C] repeated over the batch, then CorrectCone [B,S2,C]); rows are b*S+s."""
    B = len(y)
    parts = []
    if uniform_draws is not None and uniform_draws.shape[0] > 0:
        u = uniform_simplex(uniform_draws)
        parts.append(np.broadcast_to(u[None], (B,) + u.shape))
    if cone_draws is not None and cone_draws.shape[1] > 0:
        parts.append(correct_cone(cone_draws, y))
    h = np.concatenate(parts, axis=1)
    return np.ascontiguousarray(h.reshape(-1, h.shape[-1]), dtype=F32)


# ---------------------------------------------------------------------------------------------
# Cayley parametrisation (public ortho-conv design; the reference's libs/ortho_conv is an empty
# submodule, its in-tree statement is classification.py:281-294).  parity unpinned.
# ---------------------------------------------------------------------------------------------

def cayley(W: np.ndarray) -> np.ndarray:
    """Q = cayley(W) for W [cout, cin]: if cin > cout, transpose; U=W[:cin], V=W[cin:],
    A = U - U^T + V^T V, Q = [(I+A)^-1 (I-A); -2 V (I+A)^-1].  Float64 internally."""
    W = np.asarray(W, dtype=np.float64)
    cout, cin = W.shape
    if cin > cout:
        return cayley(W.T).T
    U, V = W[:cin], W[cin:]
    I = np.eye(cin)
    A = U - U.T + V.T @ V
    inv = np.linalg.inv(I + A)
    return np.concatenate([inv @ (I - A), -2.0 * V @ inv], axis=0)


def cayley_linear_weight(W: np.ndarray, alpha: float) -> np.ndarray:
    """``CayleyLinear`` effective weight: cayley(alpha * W / ||W||_F) (classification.py:282-293)."""
    W = np.asarray(W, dtype=np.float64)
    return cayley(alpha * W / np.linalg.norm(W)).astype(F32)


# ---------------------------------------------------------------------------------------------
# Dynamics -- dynamics/classification.py:96-115
# ---------------------------------------------------------------------------------------------

@dataclass
class DynParams:
    """Effective (post-Cayley) weights of ``OrthoClassDynProjectSimplexLips``; nn.Linear layout
    [out, in].  hidden_to_mlp=Q1 [M,C], U_x=Qx [M,X], mlp_to_mlp=Q2 [M,M], mlp_to_hidden=Q3 [C,M]."""
    Q1: np.ndarray
    b1: np.ndarray
    Qx: np.ndarray
    bx: np.ndarray
    Q2: np.ndarray
    b2: np.ndarray
    Q3: np.ndarray
    b3: np.ndarray

    def astype32(self) -> "DynParams":
        return DynParams(*[np.ascontiguousarray(getattr(self, k), dtype=F32) for k in
                           ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")])


@dataclass
class DynConfig:
    """Constructor fields of ``OrthoClassDynProjectSimplexLips`` that the hot path reads
    (classification.py:32-66; README.md:27 values as defaults)."""
    alpha_1: float = 100.0
    alpha_2: float = 20.0
    sigma_1: float = 0.02
    scale_nominal: bool = True
    dropout: float = 0.5
    qp_max_iter: int = 30
    qp_tol: float = 1e-4


def static_projection(x: np.ndarray, P: DynParams) -> np.ndarray:
    """Per-image term of the first layer: U_x(x) = x Qx^T + bx  -> [B, M]."""
    return (np.asarray(x, np.float64) @ P.Qx.astype(np.float64).T + P.bx).astype(F32)


def mlp_forward(h: np.ndarray, u_rows: np.ndarray, P: DynParams, mask1: Optional[np.ndarray],
                mask2: Optional[np.ndarray], p: float) -> Dict[str, np.ndarray]:
    """``_h_dot_raw`` (classification.py:96-102) with dropout given as keep-masks (uint8 0/1):
    z1 = hidden_to_mlp(h) + U_x(x); a1 = relu(drop(z1)); z2 = mlp_to_mlp(a1);
    a2 = relu(drop(z2)); ftilde = mlp_to_hidden(a2).  ``u_rows`` = U_x(x) expanded to rows.
    Matmuls in float64, activations rounded to float32 (the device accumulates in float32)."""
    scale = F32(1.0 / (1.0 - p)) if p > 0 else F32(1.0)
    h64 = np.asarray(h, np.float64)
    z1 = ((h64 @ P.Q1.astype(np.float64).T + P.b1).astype(F32) + u_rows).astype(F32)
    d1 = z1 * (mask1.astype(F32) * scale) if mask1 is not None else z1
    a1 = np.maximum(d1, F32(0)).astype(F32)
    z2 = (a1.astype(np.float64) @ P.Q2.astype(np.float64).T + P.b2).astype(F32)
    d2 = z2 * (mask2.astype(F32) * scale) if mask2 is not None else z2
    a2 = np.maximum(d2, F32(0)).astype(F32)
    ft = (a2.astype(np.float64) @ P.Q3.astype(np.float64).T + P.b3).astype(F32)
    return dict(z1=z1, a1=a1, z2=z2, a2=a2, ftilde=ft)


def barrier_lower(h: np.ndarray, cfg: DynConfig) -> np.ndarray:
    """lower = -alpha_1 * (exp(sigma_1 * h) - 1)   (classification.py:108)."""
    h = np.asarray(h, F32)
    return (F32(-cfg.alpha_1) * (np.exp(F32(cfg.sigma_1) * h).astype(F32) - F32(1))).astype(F32)


def barrier_upper(h: np.ndarray, cfg: DynConfig) -> np.ndarray:
    """upper = alpha_2 * (1 - h)   (classification.py:109)."""
    return (F32(cfg.alpha_2) * (F32(1) - np.asarray(h, F32))).astype(F32)


def sigmoid32(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float64)
    return (1.0 / (1.0 + np.exp(-x))).astype(F32)


def scale_nominal(ftilde: np.ndarray, lower: np.ndarray, upper: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """(upper - lower) * sigmoid(ftilde) + lower   (classification.py:110-112); returns
    (nominal, sigmoid) -- the sigmoid is kept for the backward."""
    sig = sigmoid32(ftilde)
    return (((upper - lower).astype(F32) * sig).astype(F32) + lower).astype(F32), sig


# ---------------------------------------------------------------------------------------------
# QP -- barrier_projection/barrier_projection.py:217-313 (FastBarrierProjectionNoUpper)
# ---------------------------------------------------------------------------------------------

@dataclass
class QPResult:
    v: np.ndarray             # [N, C] projected velocity
    mu: np.ndarray            # [N] dual variable at the exit iteration
    iters: int                # index of the exit iteration (0-based); max_iter-1 if no exit
    converged: bool
    conv_mask: np.ndarray     # [N] uint32: bit i set iff |eps_i| < tol for that row


def row_sum_seq(v: np.ndarray) -> np.ndarray:
    """Sequential left-to-right float32 sum over the last axis."""
    s = np.zeros(v.shape[:-1], dtype=F32)
    for j in range(v.shape[-1]):
        s = (s + v[..., j]).astype(F32)
    return s


def qp_forward(lower: np.ndarray, nominal: np.ndarray, max_iter: int = 30, tol: float = 1e-4) -> QPResult:
    """Bisection on mu for argmin ||v - nominal||^2 s.t. sum v = 0, v >= lower
    (barrier_projection.py:220-269).  Bracket [min nominal, max(nominal - lower)] (:232-234);
    mu = (ceil - floor)/2 + floor; v = max(nominal - mu, lower); eps = sum v (:241-246).
    BATCH-GLOBAL exit: stop every row at the first iteration where max|eps| < tol (:247-249);
    otherwise eps>0 raises the floor, eps<0 lowers the ceiling (:251-255)."""
    lower = np.asarray(lower, F32)
    nominal = np.asarray(nominal, F32)
    N = nominal.shape[0]
    mu_ceil = (nominal - lower).astype(F32).max(axis=1)
    mu_floor = nominal.min(axis=1)
    conv = np.zeros(N, dtype=np.uint32)
    tol32 = F32(tol)
    v = np.zeros_like(nominal)
    mu = np.zeros(N, F32)
    exit_iter, converged = max_iter - 1, False
    for i in range(max_iter):
        mu = ((mu_ceil - mu_floor).astype(F32) / F32(2) + mu_floor).astype(F32)
        v = np.maximum((nominal - mu[:, None]).astype(F32), lower)
        eps = row_sum_seq(v)
        ok = np.abs(eps) < tol32
        conv |= (ok.astype(np.uint32) << np.uint32(i))
        if N == 0 or bool(ok.all()):
            exit_iter, converged = i, True
            break
        mu_floor = np.where(eps > 0, mu, mu_floor).astype(F32)
        mu_ceil = np.where(eps < 0, mu, mu_ceil).astype(F32)
    # rows keep bisecting after the exit in the device's pass 1; record the full mask too
    if converged:
        conv = qp_convergence_masks(lower, nominal, max_iter, tol)
    return QPResult(v=v.astype(F32), mu=mu.astype(F32), iters=exit_iter, converged=converged,
                    conv_mask=conv)


def qp_convergence_masks(lower: np.ndarray, nominal: np.ndarray, max_iter: int = 30,
                         tol: float = 1e-4) -> np.ndarray:
    """Per-row 30-bit masks of the iterations at which the row alone meets tol, running all
    ``max_iter`` iterations (each row's bisection path is independent of the others)."""
    lower = np.asarray(lower, F32)
    nominal = np.asarray(nominal, F32)
    mu_ceil = (nominal - lower).astype(F32).max(axis=1)
    mu_floor = nominal.min(axis=1)
    conv = np.zeros(nominal.shape[0], dtype=np.uint32)
    for i in range(max_iter):
        mu = ((mu_ceil - mu_floor).astype(F32) / F32(2) + mu_floor).astype(F32)
        v = np.maximum((nominal - mu[:, None]).astype(F32), lower)
        eps = row_sum_seq(v)
        conv |= ((np.abs(eps) < F32(tol)).astype(np.uint32) << np.uint32(i))
        mu_floor = np.where(eps > 0, mu, mu_floor).astype(F32)
        mu_ceil = np.where(eps < 0, mu, mu_ceil).astype(F32)
    return conv


def global_exit_iteration(conv_masks: np.ndarray, max_iter: int = 30) -> int:
    """Lowest iteration at which every row meets tol, else max_iter-1 (no exit)."""
    m = np.uint32((1 << max_iter) - 1)
    for c in np.asarray(conv_masks, np.uint32).ravel():
        m &= c
    if m == 0:
        return max_iter - 1
    return int((int(m) & -int(m)).bit_length() - 1)


def qp_run_fixed(lower: np.ndarray, nominal: np.ndarray, iters: int) -> Tuple[np.ndarray, np.ndarray]:
    """Run exactly iters+1 bisection steps (iteration indices 0..iters); return (v, mu) of the
    last one -- the state the reference returns when it exits at ``iters``."""
    lower = np.asarray(lower, F32)
    nominal = np.asarray(nominal, F32)
    mu_ceil = (nominal - lower).astype(F32).max(axis=1)
    mu_floor = nominal.min(axis=1)
    v = mu = None
    for i in range(iters + 1):
        mu = ((mu_ceil - mu_floor).astype(F32) / F32(2) + mu_floor).astype(F32)
        v = np.maximum((nominal - mu[:, None]).astype(F32), lower)
        eps = row_sum_seq(v)
        mu_floor = np.where(eps > 0, mu, mu_floor).astype(F32)
        mu_ceil = np.where(eps < 0, mu, mu_ceil).astype(F32)
    return v.astype(F32), mu.astype(F32)


def qp_backward(g: np.ndarray, v: np.ndarray, mu: np.ndarray, lower: np.ndarray,
                nominal: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Closed form of the dense-Jacobian backward (barrier_projection.py:271-311).
    lambda = (v - nominal) + mu; active = lambda > 0; na = ~active; r = 1/|na| (float32);
    g_nominal[j] = na_j * (g_j - r * sum_{i in na} g_i)
    g_lower[j]   = act_j * (g_j - r * sum_{i in na} g_i)
    With |na| = 0 the reference's masked_scatter touches nothing: g_nominal = 0, g_lower = g."""
    g = np.asarray(g, F32)
    lam = ((np.asarray(v, F32) - np.asarray(nominal, F32)).astype(F32) + np.asarray(mu, F32)[:, None]).astype(F32)
    act = lam > 0
    na = ~act
    card = na.sum(axis=1)
    s = row_sum_seq(np.where(na, g, F32(0)).astype(F32))
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(card > 0, F32(1) / np.maximum(card, 1).astype(F32), F32(0)).astype(F32)
    corr = (r * s).astype(F32)[:, None]
    d = (g - corr).astype(F32)
    g_nom = np.where(na, d, F32(0)).astype(F32)
    g_low = np.where(act, d, F32(0)).astype(F32)
    return g_low, g_nom


# ---------------------------------------------------------------------------------------------
# eval_dot -- classification.py:104-126
# ---------------------------------------------------------------------------------------------

@dataclass
class EvalDotResult:
    f: np.ndarray
    ftilde: np.ndarray      # raw MLP output
    nominal: np.ndarray     # after optional sigmoid scaling
    sig: Optional[np.ndarray]
    lower: np.ndarray
    qp: QPResult
    mlp: Dict[str, np.ndarray]


def eval_dot(h: np.ndarray, u_rows: np.ndarray, P: DynParams, cfg: DynConfig,
             mask1: Optional[np.ndarray] = None, mask2: Optional[np.ndarray] = None,
             p: Optional[float] = None, qp_inputs: Optional[Tuple[np.ndarray, np.ndarray]] = None) -> EvalDotResult:
    """``eval_dot`` / ``eval_dot_light`` (classification.py:104-126).  Masks None = eval mode.

    ``qp_inputs`` = (lower, nominal) pins the QP inputs to another implementation's float32
    values.  The reference's QP backward decides its active set by the sign of
    ``(v - nominal) + mu`` (barrier_projection.py:288-289), which for an inactive coordinate is
    pure float32 rounding noise; two implementations whose MLPs differ in the last bit therefore
    pick different active sets.  Stage-wise parity checks pin the QP inputs to compare the rest."""
    p = cfg.dropout if p is None else p
    mlp = mlp_forward(h, u_rows, P, mask1, mask2, p if mask1 is not None else 0.0)
    lower = barrier_lower(h, cfg)
    if cfg.scale_nominal:
        nominal, sig = scale_nominal(mlp["ftilde"], lower, barrier_upper(h, cfg))
    else:
        nominal, sig = mlp["ftilde"], None
    if qp_inputs is not None:
        lower = np.asarray(qp_inputs[0], F32)
        nominal = np.asarray(qp_inputs[1], F32)
    qp = qp_forward(lower, nominal, cfg.qp_max_iter, cfg.qp_tol)
    return EvalDotResult(f=qp.v, ftilde=mlp["ftilde"], nominal=nominal, sig=sig, lower=lower, qp=qp, mlp=mlp)


# ---------------------------------------------------------------------------------------------
# DecisionBoundary V and Vdot -- lya_cands.py:79-94; pl_modules.py:403-412
# ---------------------------------------------------------------------------------------------

def runner_up(h: np.ndarray, y_rows: np.ndarray) -> np.ndarray:
    """j* = first-index argmax over the wrong classes (masked_select keeps class order)."""
    hw = np.asarray(h, F32).copy()
    np.put_along_axis(hw, np.asarray(y_rows)[:, None], -np.inf, 1)
    return np.argmax(hw, axis=1)


def decision_boundary_V(h: np.ndarray, y_rows: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """V = (1 + max_{j != y} h_j) - h_y (simplex mode, log_mode False).  Returns (V, j*)."""
    h = np.asarray(h, F32)
    js = runner_up(h, y_rows)
    hmax = np.take_along_axis(h, js[:, None], 1)[:, 0]
    hy = np.take_along_axis(h, np.asarray(y_rows)[:, None], 1)[:, 0]
    return ((F32(1) + hmax).astype(F32) - hy).astype(F32), js


def vdot(f: np.ndarray, y_rows: np.ndarray, js: np.ndarray) -> np.ndarray:
    """jvp(V, h; f) with V piecewise linear: Vdot = f[j*] - f[y]."""
    f = np.asarray(f, F32)
    return (np.take_along_axis(f, js[:, None], 1)[:, 0] -
            np.take_along_axis(f, np.asarray(y_rows)[:, None], 1)[:, 0]).astype(F32)


# ---------------------------------------------------------------------------------------------
# The training step hot path: LyapunovLearning.compute_loss (pl_modules.py:390-502) + backward
# ---------------------------------------------------------------------------------------------

@dataclass
class StepInputs:
    x_feat: np.ndarray          # [B, X] static features (backbone output)
    y: np.ndarray               # [B] labels
    h: np.ndarray               # [N, C] samples, row = b*S + s
    S: int
    mask1: Optional[np.ndarray] = None   # loss pass keep masks [N, M] uint8
    mask2: Optional[np.ndarray] = None
    lmask1: Optional[np.ndarray] = None  # logging pass keep masks
    lmask2: Optional[np.ndarray] = None
    kappa: float = 2.0
    qp_inputs: Optional[Tuple[np.ndarray, np.ndarray]] = None      # pin (lower, nominal), loss pass
    qp_inputs_log: Optional[Tuple[np.ndarray, np.ndarray]] = None  # pin (lower, nominal), logging pass


@dataclass
class StepOutputs:
    loss: float
    eff: int
    mean_active: float
    V: np.ndarray
    Vdot: np.ndarray
    viol: np.ndarray
    f: np.ndarray
    ftilde: np.ndarray
    f_log: np.ndarray
    qp_iters: int
    qp_iters_log: int
    grads: Dict[str, np.ndarray] = field(default_factory=dict)


def lyapunov_step(inp: StepInputs, P: DynParams, cfg: DynConfig) -> StepOutputs:
    """Forward (pl_modules.py:394-484) and the parameter gradients of ``loss.backward()`` w.r.t.
    the effective weights Q*, biases and the static features (act='relu', order=1)."""
    N, C = inp.h.shape
    B = inp.x_feat.shape[0]
    S = inp.S
    assert N == B * S
    y_rows = np.repeat(np.asarray(inp.y, np.int64), S)
    u = static_projection(inp.x_feat, P)                       # [B, M]
    u_rows = np.repeat(u, S, axis=0)
    ev = eval_dot(inp.h, u_rows, P, cfg, inp.mask1, inp.mask2, qp_inputs=inp.qp_inputs)
    V, js = decision_boundary_V(inp.h, y_rows)
    Vd = vdot(ev.f, y_rows, js)
    pre = (Vd + (F32(inp.kappa) * V).astype(F32)).astype(F32)
    viol = np.maximum(pre, F32(0)).astype(F32)
    loss = float(np.sum(viol, dtype=np.float64) / N)
    eff = int((viol > 0).sum())

    # logging pass (pl_modules.py:474-483): fresh dropout, *linear* lower bound in the mask test
    evl = eval_dot(inp.h, u_rows, P, cfg, inp.lmask1, inp.lmask2, qp_inputs=inp.qp_inputs_log)
    lin_lower = (F32(-cfg.alpha_1) * np.asarray(inp.h, F32)).astype(F32)
    upper = barrier_upper(inp.h, cfg)
    act = (np.abs((evl.f - lin_lower).astype(F32)) <= F32(1e-6)) | (np.abs((evl.f - upper).astype(F32)) <= F32(1e-6))
    mean_active = float(act.mean())

    # ---- backward: d mean(relu(pre)) ----
    g_pre = np.where(pre > 0, F32(1.0 / N), F32(0)).astype(F32)
    g_f = np.zeros((N, C), F32)
    np.put_along_axis(g_f, js[:, None], g_pre[:, None], 1)
    np.put_along_axis(g_f, y_rows[:, None], -g_pre[:, None], 1)
    _, g_nom = qp_backward(g_f, ev.f, ev.qp.mu, ev.lower, ev.nominal)
    if cfg.scale_nominal:
        span = (barrier_upper(inp.h, cfg) - ev.lower).astype(F32)
        g_ft = ((g_nom * span).astype(F32) * ((F32(1) - ev.sig) * ev.sig).astype(F32)).astype(F32)
    else:
        g_ft = g_nom
    grads = mlp_backward(g_ft, inp.h, inp.x_feat, S, P, ev.mlp, inp.mask1, inp.mask2, cfg.dropout)
    return StepOutputs(loss=loss, eff=eff, mean_active=mean_active, V=V, Vdot=Vd, viol=viol,
                       f=ev.f, ftilde=ev.ftilde, f_log=evl.f, qp_iters=ev.qp.iters,
                       qp_iters_log=evl.qp.iters, grads=grads)


def mlp_backward(g_ft: np.ndarray, h: np.ndarray, x_feat: np.ndarray, S: int, P: DynParams,
                 mlp: Dict[str, np.ndarray], mask1, mask2, p: float) -> Dict[str, np.ndarray]:
    """Backward of _h_dot_raw (F.linear / dropout / relu autograd rules), float64 sums."""
    scale = (1.0 / (1.0 - p)) if (p > 0 and mask1 is not None) else 1.0
    g3 = np.asarray(g_ft, np.float64)
    a1 = mlp["a1"].astype(np.float64)
    a2 = mlp["a2"].astype(np.float64)
    out = {}
    out["Q3"] = g3.T @ a2
    out["b3"] = g3.sum(0)
    g_a2 = g3 @ P.Q3.astype(np.float64)
    m2 = (mask2.astype(np.float64) * scale) if mask2 is not None else 1.0
    g_z2 = g_a2 * (mlp["a2"] > 0) * m2
    out["Q2"] = g_z2.T @ a1
    out["b2"] = g_z2.sum(0)
    g_a1 = g_z2 @ P.Q2.astype(np.float64)
    m1 = (mask1.astype(np.float64) * scale) if mask1 is not None else 1.0
    g_z1 = g_a1 * (mlp["a1"] > 0) * m1
    out["Q1"] = g_z1.T @ np.asarray(h, np.float64)
    out["b1"] = g_z1.sum(0)
    B = x_feat.shape[0]
    g_u = g_z1.reshape(B, S, -1).sum(1)                      # expand backward (pl_modules.py:400)
    out["Qx"] = g_u.T @ np.asarray(x_feat, np.float64)
    out["bx"] = g_u.sum(0)
    out["x_feat"] = g_u @ P.Qx.astype(np.float64)
    out["g_u"] = g_u
    return {k: v.astype(F32) for k, v in out.items()}


# ---------------------------------------------------------------------------------------------
# ODE solves -- torchdiffeq 0.2.2 semantics (external dependency, pinned in env.yml:251; its
# source is not in the container: restated from its published algorithm).  f(h) = eval_dot in
# eval mode (no dropout) with the QP's batch-global exit evaluated over the whole batch.
# ---------------------------------------------------------------------------------------------

def make_ode_func(x_feat: np.ndarray, P: DynParams, cfg: DynConfig, counter: Optional[list] = None):
    u = static_projection(x_feat, P)

    def func(t, h):
        if counter is not None:
            counter[0] += 1
        return eval_dot(h, u, P, cfg).f
    return func


def linspace32(t0: float, t1: float, steps: int) -> np.ndarray:
    """torch.linspace(t0, t1, steps) in float32 (the reference builds ts this way,
    pl_modules.py:323): start + i*step for the first half, end - (steps-1-i)*step after."""
    if steps == 1:
        return np.array([t0], np.float32)
    a, b = F32(t0), F32(t1)
    step = F32((b - a) / F32(steps - 1))
    out = np.empty(steps, np.float32)
    half = steps // 2
    for i in range(steps):
        out[i] = F32(a + step * F32(i)) if i < half else F32(b - step * F32(steps - 1 - i))
    return out


def rk4_grid(t0: float, t1: float, step_size: float) -> np.ndarray:
    """FixedGridODESolver._grid_constructor_from_step_size in float32 (the reference's ts are
    float32): niters = ceil((t1-t0)/h + 1); t_k = k*h + t0; last point snapped to t1."""
    a, b, h = F32(t0), F32(t1), F32(step_size)
    niters = int(math.ceil(float(F32(F32(b - a) / h) + F32(1))))
    grid = (np.arange(niters, dtype=np.float32) * h + a).astype(np.float32)
    grid[-1] = b
    return grid


def rk4_fixed_grid(func, y0: np.ndarray, t0: float, t1: float, step_size: float,
                   times: Optional[np.ndarray] = None):
    """torchdiffeq method='rk4' (FixedGridODESolver + rk4_alt_step_func, the 3/8 rule) with
    ``options.step_size`` (pl_modules.py:27-33).  Returns (solution at ``times`` [T,B,C] -- or
    y(t1) when times is None --, number of steps).  Output points use the solver's linear
    interpolation (exact grid hits return the grid value)."""
    y = np.asarray(y0, F32)
    grid = rk4_grid(t0, t1, step_size)
    ts = np.array([t0, t1], np.float32) if times is None else np.asarray(times, np.float32)
    sol = [y.copy()]
    j = 1
    third = F32(1.0 / 3.0)
    for a, b in zip(grid[:-1], grid[1:]):
        dt = F32(b - a)
        k1 = func(float(a), y)
        k2 = func(float(a + dt * third), (y + (dt * k1).astype(F32) * third).astype(F32))
        k3 = func(float(a + dt * F32(2.0 / 3.0)), (y + dt * (k2 - (k1 * third).astype(F32)).astype(F32)).astype(F32))
        k4 = func(float(b), (y + dt * ((k1 - k2).astype(F32) + k3).astype(F32)).astype(F32))
        dy = ((((k1 + F32(3) * (k2 + k3).astype(F32)).astype(F32) + k4).astype(F32) * dt).astype(F32) * F32(0.125)).astype(F32)
        y1 = (y + dy).astype(F32)
        while j < len(ts) and b >= ts[j]:
            if ts[j] == a:
                sol.append(y.copy())
            elif ts[j] == b:
                sol.append(y1.copy())
            else:
                slope = F32((ts[j] - a) / (b - a))
                sol.append((y + slope * (y1 - y).astype(F32)).astype(F32))
            j += 1
        y = y1
    if times is None:
        return y, len(grid) - 1
    return np.stack(sol), len(grid) - 1


def rk4_on_grid(func, y0: np.ndarray, grid: np.ndarray) -> np.ndarray:
    """torchdiffeq method='rk4' WITHOUT options.step_size: the solver grid is the output times
    themselves (FixedGridODESolver's default grid constructor), so the solution is the grid
    states [T, ...] -- the call of BASELINE configs[0] (control/certify_segway.py:108-109,
    ts = linspace(0, 50, 10000)).  Same float32 3/8-rule expressions as rk4_fixed_grid."""
    y = np.asarray(y0, F32)
    g = np.asarray(grid, F32)
    third = F32(1.0 / 3.0)
    sol = [y.copy()]
    for a, b in zip(g[:-1], g[1:]):
        dt = F32(b - a)
        k1 = np.asarray(func(float(a), y), F32)
        k2 = np.asarray(func(float(a + dt * third), (y + (dt * k1).astype(F32) * third).astype(F32)), F32)
        k3 = np.asarray(func(float(a + dt * F32(2.0 / 3.0)),
                             (y + dt * (k2 - (k1 * third).astype(F32)).astype(F32)).astype(F32)), F32)
        k4 = np.asarray(func(float(b), (y + dt * ((k1 - k2).astype(F32) + k3).astype(F32)).astype(F32)), F32)
        dy = ((((k1 + F32(3) * (k2 + k3).astype(F32)).astype(F32) + k4).astype(F32) * dt).astype(F32)
              * F32(0.125)).astype(F32)
        y = (y + dy).astype(F32)
        sol.append(y.copy())
    return np.stack(sol)


def rk4_train(x_feat: np.ndarray, h0: np.ndarray, P: DynParams, cfg: DynConfig, t0: float, t1: float,
              step_size: float, masks: Optional[np.ndarray] = None, p: Optional[float] = None):
    """The train_ode forward (pl_modules.py:490-493): odeint with method='rk4' and the dynamics in
    TRAIN mode -- every func() call is eval_dot with its own dropout masks ``masks[e]`` =
    (layer-1, layer-2) keep masks of eval e, [E,2,B,M] uint8 (None = eval mode).  Returns
    (y(t1), records) with records[e] = (stage input h, EvalDotResult)."""
    u = static_projection(x_feat, P)
    recs = []

    def func(t, h):
        e = len(recs)
        m1, m2 = (masks[e, 0], masks[e, 1]) if masks is not None else (None, None)
        r = eval_dot(h, u, P, cfg, m1, m2, p)
        recs.append((np.asarray(h, F32).copy(), r))
        return r.f
    y, _ = rk4_fixed_grid(func, h0, t0, t1, step_size)
    return y, recs


DOPRI5_ALPHA = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0]
DOPRI5_BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
DOPRI5_C_ERROR = [
    35 / 384 - 1951 / 21600, 0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
    -2187 / 6784 - -12231 / 42400, 11 / 84 - 649 / 6300, -1.0 / 60.0,
]
DOPRI5_C_MID = [
    6025192743 / 30085553152 / 2, 0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
    187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2,
]


def rms_norm(x: np.ndarray) -> F32:
    """torchdiffeq ``_rms_norm`` (= ``_mixed_norm`` on a 1-tuple): sqrt(mean(x^2)) over the whole
    batch -- ONE error norm shared by every sample."""
    x = np.asarray(x, F32)
    return F32(math.sqrt(float(np.mean(np.square(x.astype(np.float64))))))


@dataclass
class Dopri5Stats:
    nfe: int = 0
    n_accept: int = 0
    n_reject: int = 0
    steps: List[Tuple[float, float, bool, float]] = field(default_factory=list)


def dopri5(func, y0: np.ndarray, t0: float, t1: float, rtol: float, atol: float,
           safety: float = 0.9, ifactor: float = 10.0, dfactor: float = 0.2,
           max_steps: int = 100000, times: Optional[np.ndarray] = None) -> Tuple[np.ndarray, Dopri5Stats]:
    """torchdiffeq 0.2.2 RKAdaptiveStepsizeODESolver with the Dormand-Prince tableau: initial
    step from _select_initial_step(order-1=4), FSAL stages, batch-global RMS error ratio,
    accept iff ratio <= 1, _optimal_step_size(order 5), dense output at t1 by the 4th-order
    interpolant fitted with DPS_C_MID.  Times float64, state float32."""
    st = Dopri5Stats()
    y = np.asarray(y0, F32)
    rtol32, atol32 = F32(rtol), F32(atol)
    f0 = func(t0, y); st.nfe += 1
    # _select_initial_step (float32)
    scale = (atol32 + np.abs(y) * rtol32).astype(F32)
    d0 = rms_norm(y / scale)
    d1 = rms_norm(f0 / scale)
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = F32(1e-6)
    else:
        h0 = F32(F32(0.01) * d0 / d1)
    y1 = (y + h0 * f0).astype(F32)
    f1 = func(t0 + float(h0), y1); st.nfe += 1
    d2 = F32(rms_norm((f1 - f0).astype(F32) / scale) / h0)
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = max(F32(1e-6), F32(h0 * F32(1e-3)))
    else:
        h1 = F32(F32(0.01) / max(d1, d2)) ** F32(1.0 / 5.0)
    dt = float(min(F32(100) * h0, F32(h1)))
    beta = [np.asarray(b, F32) for b in DOPRI5_BETA]
    cerr = np.asarray(DOPRI5_C_ERROR, F32)
    cmid = np.asarray(DOPRI5_C_MID, F32)
    tcur = t0
    fcur = f0
    interp = None
    tprev, tnext = t0, t0
    ts = [t0, t1] if times is None else [float(t) for t in times]
    sol = [y.copy()]
    for tout in ts[1:]:
        while tout > tnext:
            if len(st.steps) >= max_steps:
                raise RuntimeError("dopri5: too many steps")
            assert tcur + dt > tcur, "underflow in dt"
            ta = tcur + dt
            dt32 = F32(dt)
            k = [fcur]
            for i in range(6):
                coeffs = (beta[i] * dt32).astype(F32)
                acc = np.zeros_like(y)
                for j in range(i + 1):
                    acc = (acc + k[j] * coeffs[j]).astype(F32)
                yi = (y + acc).astype(F32)
                k.append(func(ta if DOPRI5_ALPHA[i] == 1.0 else tcur + DOPRI5_ALPHA[i] * dt, yi)); st.nfe += 1
            ynew = yi
            ce = (cerr * dt32).astype(F32)
            err = np.zeros_like(y)
            for j in range(7):
                err = (err + k[j] * ce[j]).astype(F32)
            etol = (atol32 + rtol32 * np.maximum(np.abs(y), np.abs(ynew))).astype(F32)
            ratio = rms_norm((err / etol).astype(F32))
            accept = ratio <= 1
            st.steps.append((tcur, dt, bool(accept), float(ratio)))
            if accept:
                cm = (cmid * dt32).astype(F32)
                acc = np.zeros_like(y)
                for j in range(7):
                    acc = (acc + k[j] * cm[j]).astype(F32)
                ymid = (y + acc).astype(F32)
                fa, fb = k[0], k[6]
                a = (F32(2) * dt32 * (fb - fa) - F32(8) * (ynew + y) + F32(16) * ymid).astype(F32)
                b = (dt32 * (F32(5) * fa - F32(3) * fb) + F32(18) * y + F32(14) * ynew - F32(32) * ymid).astype(F32)
                c = (dt32 * (fb - F32(4) * fa) - F32(11) * y - F32(5) * ynew + F32(16) * ymid).astype(F32)
                d = (dt32 * fa).astype(F32)
                interp = [y.copy(), d, c, b, a]
                tprev, tnext = tcur, ta
                y, fcur, tcur = ynew, k[6], ta
                st.n_accept += 1
            else:
                st.n_reject += 1
            # _optimal_step_size (float64)
            if ratio == 0:
                dt = dt * ifactor
            else:
                df = 1.0 if ratio < 1 else dfactor
                dt = dt * min(ifactor, max(safety / float(ratio) ** (1.0 / 5.0), df))
        x = F32((tout - tprev) / (tnext - tprev))
        total = (interp[0] + x * interp[1]).astype(F32)
        xp = x
        for coef in interp[2:]:
            xp = F32(xp * x)
            total = (total + xp * coef).astype(F32)
        sol.append(total)
    if times is None:
        return sol[-1], st
    return np.stack(sol), st


# ---------------------------------------------------------------------------------------------
# Certification grid -- robustness/eval_utils.py:31-89, robustness/certify_lipschitz.py:37-143
# ---------------------------------------------------------------------------------------------

def db_count_table(n: int = 10, T: int = 40) -> List[List[int]]:
    """Row counts of the decision-boundary grid construction (count_samples_decision_boundary,
    eval_utils.py:72-89): f[j][k] = number of k-dim non-negative integer vectors with sum j whose
    coordinate 0 equals the max of the others, in the construction's case split."""
    f = [[0] * (n + 1) for _ in range(T + 1)]
    for j in range(T + 1):
        for k in range(n + 1):
            if j == 0:
                f[j][k] = 1
            elif k < 2 or j == 1:
                f[j][k] = 0
            elif k == 2:
                f[j][k] = 1 if j % 2 == 0 else 0
            else:
                f[j][k] = sum(f[j - k + l][k - l] * math.comb(k - 1, l)
                              for l in range(k - 1) if j - k + l >= 0)
    return f


def db_grid_rows(n: int, T: int) -> np.ndarray:
    """The grid of sample_decision_boundary (eval_utils.py:31-61) as integer vectors v (eta = v/T),
    in the construction's row order: for a (sum j, dim k) block, rows are grouped by the number l
    of zero coordinates among 1..k-1, then by the lexicographic position set c of the non-zero
    ones, then by the row order of the (sum j-k+l, dim k-l) sub-block plus one."""
    memo = {}

    def block(j, k):
        key = (j, k)
        if key in memo:
            return memo[key]
        if j == 0:
            out = np.zeros((1, k), np.int64)
        elif k < 2 or j == 1:
            out = np.zeros((0, k), np.int64)
        elif k == 2:
            out = np.array([[j // 2, j // 2]], np.int64) if j % 2 == 0 else np.zeros((0, 2), np.int64)
        else:
            parts = []
            for l in range(k - 1):
                if j - k + l < 0:
                    continue
                sub = block(j - k + l, k - l) + 1
                for c in __import__("itertools").combinations(range(1, k), k - l - 1):
                    rows = np.zeros((sub.shape[0], k), np.int64)
                    rows[:, [0] + list(c)] = sub
                    parts.append(rows)
            out = np.concatenate(parts) if parts else np.zeros((0, k), np.int64)
        memo[key] = out
        return out

    return block(T, n)


def db_unrank(r: int, n: int, T: int, f: List[List[int]]) -> List[int]:
    """Row r of db_grid_rows(n, T) without materialising the grid (what the device kernel does)."""
    out = [0] * n
    idx = list(range(n))
    add, j, k = 0, T, n
    while True:
        if j == 0:
            for p in idx:
                out[p] = add
            return out
        if k == 2:
            out[idx[0]] = out[idx[1]] = add + j // 2
            return out
        for l in range(k - 1):
            if j - k + l < 0:
                continue
            sub = f[j - k + l][k - l]
            blk = math.comb(k - 1, k - l - 1) * sub
            if r < blk:
                break
            r -= blk
        m = k - l - 1
        ci, r = divmod(r, sub)
        c, e = [], 1
        while len(c) < m:                      # lexicographic combination unranking over 1..k-1
            cnt = math.comb(k - 1 - e, m - len(c) - 1)
            if ci < cnt:
                c.append(e)
            else:
                ci -= cnt
            e += 1
        keep = [0] + c
        for p in range(k):
            if p not in keep:
                out[idx[p]] = add
        idx = [idx[p] for p in keep]
        add, j, k = add + 1, j - k + l, k - l


def db_grid_for_label(grid_v: np.ndarray, label: int, T: int) -> np.ndarray:
    """get_grid_for_label (eval_utils.py:64-69): swap columns 0 and label; eta = v / T as float32."""
    g = np.asarray(grid_v, np.float64) / T
    if label != 0:
        g[:, [label, 0]] = g[:, [0, label]]
    return g.astype(F32)


@dataclass
class CertifyConst:
    T: int = 40
    n: int = 10
    eps_cfg: float = 0.141          # cfg.eps (CertifyExpCfg, ExpConfig.py:353)
    min_std: float = 0.225          # min(param_map[0].std)
    batches: int = 10

    def kappa(self, cfg: DynConfig) -> float:
        lfx = (cfg.alpha_1 if cfg.scale_nominal else 1.0) / self.min_std   # certify_lipschitz.py:67-70
        return math.sqrt(2) * lfx * self.eps_cfg                              # :72


def certify_batches(G: int, batches: int) -> List[Tuple[int, int]]:
    """certify_lipschitz.py:100-102, 115-119: ebs = G // batches, +1 batch when G % batches != 0,
    the last batch takes the tail."""
    ebs = G // batches
    nb = batches + (1 if G % batches != 0 else 0)
    out = []
    for b in range(nb):
        if (b + 1) * ebs < G:
            out.append((b * ebs, (b + 1) * ebs))
        else:
            out.append((b * ebs, G))
    return out


def certify_image(x_feat: np.ndarray, label: int, grid_v: np.ndarray, P: DynParams, cfg: DynConfig,
                  cc: CertifyConst) -> Tuple[np.ndarray, np.ndarray]:
    """Per-batch max violation and max violation_larger_T for one image (certify_lipschitz.py:104-136).
    The QP's global exit runs over each batch's rows, as eval_dot_light sees them."""
    eta_all = db_grid_for_label(grid_v, label, cc.T)
    u = static_projection(np.asarray(x_feat, F32).reshape(1, -1), P)
    eps_g = F32(1.0 / cc.T)
    dist = F32(math.sqrt(cc.n) / cc.T)
    kappa = F32(cc.kappa(cfg))
    vmax, vtmax = [], []
    for lo, hi in certify_batches(len(eta_all), cc.batches):
        eta = eta_all[lo:hi]
        if len(eta) == 0:
            continue
        ev = eval_dot(eta, np.repeat(u, len(eta), 0), P, cfg)
        f = ev.f
        ub = (eta.max(1) + eps_g).astype(F32)
        lf = ((F32(math.sqrt(cc.n)) * (F32(cfg.sigma_1 * cfg.alpha_1) * np.exp(F32(cfg.sigma_1) * ub).astype(F32)))
              .astype(F32) + F32(1)).astype(F32)
        perturb = ((F32(math.sqrt(2)) * lf).astype(F32) * dist).astype(F32)
        mx = eta.max(1, keepdims=True)
        wrong = eta == mx
        wrong[:, label] = False
        fw = np.where(wrong, f, -np.inf).max(1).astype(F32)
        hv = ((-f[:, label]).astype(F32) + fw).astype(F32)
        vmax.append(float(((hv + perturb).astype(F32) + kappa).astype(F32).max()))
        vtmax.append(float((hv + kappa).astype(F32).max()))
    return np.array(vmax, np.float32), np.array(vtmax, np.float32)
