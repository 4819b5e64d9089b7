"""Tensor-level wrappers over the C-ABI (device tensors in, device tensors out).

Every wrapper checks shapes/dtypes/devices on the host before launching (a wrong shape must
never reach a kernel), runs on the caller's current HIP stream, and caches workspaces per
(device, size).  No CPU fallback exists: the tensors must live on a ROCm device.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import _lib as L

C, M, X = 10, 128, 10
WEIGHT_KEYS = ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")
WEIGHT_SHAPES = {"Q1": (M, C), "b1": (M,), "Qx": (M, X), "bx": (M,), "Q2": (M, M), "b2": (M,),
                 "Q3": (C, M), "b3": (C,)}


@dataclass
class DynCfg:
    """Mirror of fiode_dyn_config (the dynamics constructor fields the hot path reads)."""
    alpha_1: float = 100.0
    alpha_2: float = 20.0
    sigma_1: float = 0.02
    scale_nominal: bool = True
    dropout: float = 0.5
    qp_max_iter: int = 30
    qp_tol: float = 1e-4

    def to_c(self) -> L.DynConfig:
        return L.DynConfig(C, M, X, float(self.alpha_1), float(self.alpha_2), float(self.sigma_1),
                           int(bool(self.scale_nominal)), float(self.dropout), int(self.qp_max_iter),
                           float(self.qp_tol))


def _stream(dev: torch.device) -> ct.c_void_p:
    return ct.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need(t: torch.Tensor, name: str, shape, dtype, dev) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device != dev or t.device.type != "cuda":
        raise ValueError(f"{name}: must be on {dev} (ROCm device); got {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t.contiguous()


# tools/ab_step.py `ws_fill`: zeroed workspaces made inside a capture by a captured fill (before r06)
WS_FILL_IN_CAPTURE = False


class _Workspace:
    _cache: Dict[tuple, torch.Tensor] = {}
    _arena: Dict[int, list] = {}          # device -> [buffer, slot bytes, next slot]
    _zero_max: Dict[int, int] = {}        # device -> largest zeroed workspace asked for so far
    fills_in_capture = 0                  # zeroed workspaces a capture had to fill itself
    _retired: list = []                   # buffers a larger one replaced (a captured graph may hold them)

    @classmethod
    def get(cls, dev: torch.device, nbytes: int, tag: str, zero: bool = False) -> torch.Tensor:
        """A cached device buffer of at least ``nbytes`` per (device, tag); ``zero``: a new buffer
        starts zeroed (for kernels whose flag words must be zero on first use and are left zero by
        every call).

        A zeroed buffer first asked for inside a hipGraph capture is a slot of the arena that
        ``reserve`` zeroed before the capture: memory the capture's own pool would hand out can be
        an earlier temporary of the same replay (written before this call on every replay), so a
        buffer from it would need a captured fill on the step's chain.  Without a free slot large
        enough, the capture fills (``fills_in_capture`` counts it)."""
        key = (dev.index, tag)
        buf = cls._cache.get(key)
        if zero:
            cls._zero_max[dev.index] = max(cls._zero_max.get(dev.index, 0), int(nbytes))
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                # never freed: a graph captured with it replays into its address
                cls._retired.append(buf)
            n = max(int(nbytes), 256)
            ar = cls._arena.get(dev.index)
            if (zero and not WS_FILL_IN_CAPTURE and ar is not None and ar[1] >= n and
                    (ar[2] + 1) * ar[1] <= ar[0].numel() and torch.cuda.is_current_stream_capturing()):
                buf = ar[0][ar[2] * ar[1]:(ar[2] + 1) * ar[1]]
                ar[2] += 1
            else:
                if zero and torch.cuda.is_current_stream_capturing():
                    cls.fills_in_capture += 1
                buf = (torch.zeros if zero else torch.empty)(n, dtype=torch.uint8, device=dev)
            cls._cache[key] = buf
        return buf

    @classmethod
    def reserve(cls, dev: torch.device, slots: int) -> None:
        """Before a capture (outside it): a zeroed arena of ``slots`` slots, each as large as the
        largest zeroed workspace asked for so far (the eager warm-up's), for the streams the
        capture makes.  Slots handed out earlier stay with their streams (kernels leave them zero)."""
        nb = (max(cls._zero_max.get(dev.index, 0), 256) + 255) // 256 * 256
        cls._arena[dev.index] = [torch.zeros(slots * nb, dtype=torch.uint8, device=dev), nb, 0]


def _weights_c(w: Dict[str, torch.Tensor], dev) -> tuple:
    ws = {k: _need(w[k], k, WEIGHT_SHAPES[k], torch.float32, dev) for k in WEIGHT_KEYS}
    return ws, L.DynWeights(*[ws[k].data_ptr() for k in WEIGHT_KEYS])


def sampler_draws_count(sampler: int, B: int, S: int, n_uniform: int) -> int:
    """Number of Exp(1) variates one fiode_lyap_step sampler consumes (fiode_lyap_io.exp_draws):
    COMPOSITE [S1][C] + [B][S-S1][C]; TRAJECTORY [S1][C]; DECISION_BOUNDARY [B][S][C-1]."""
    if sampler == L.FIODE_SAMPLER_COMPOSITE:
        return n_uniform * C + B * (S - n_uniform) * C
    if sampler == L.FIODE_SAMPLER_TRAJECTORY:
        return n_uniform * C
    if sampler == L.FIODE_SAMPLER_DECISION_BOUNDARY:
        return B * S * (C - 1)
    return 0


def lyap_step(x_feat: torch.Tensor, y: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg, *,
              sample_size: int, n_uniform: int, sampler: int = L.FIODE_SAMPLER_COMPOSITE,
              dropout_mode: int = L.FIODE_DROPOUT_PHILOX, kappa: float = 2.0, seed: int = 0, offset: int = 0,
              h: Optional[torch.Tensor] = None, masks: Optional[torch.Tensor] = None, debug: bool = False,
              out: Optional[dict] = None, events=None, offset_dev: Optional[torch.Tensor] = None,
              exp_draws: Optional[torch.Tensor] = None, kappa_dev: Optional[torch.Tensor] = None):
    """The fused training step (fiode_lyap_step).  Returns (scalars[8], grads dict, debug dict).
    ``events``: optional list of len(_lib.LYAP_KERNELS)+1 torch.cuda.Event(enable_timing=True),
    recorded by the library around each of its kernels on the current stream.
    ``offset_dev``: optional int64 [1] device tensor added to ``offset`` by the kernels (a captured
    graph of the step advances it on every replay).
    ``exp_draws``: optional flat float32 Exp(1) variates for the sampler (``sampler_draws_count``
    of them, the reference's draw shapes) instead of the in-kernel Philox draws.
    ``debug``: also returns the per-row outputs, the Exp(1) variates the sampler used
    (``exp_draws``) and the dropout keep words (``keep_words`` int32 [4, N, 4])."""
    dev = x_feat.device
    B = x_feat.shape[0]
    S = int(sample_size)
    N = B * S
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    y = _need(y, "y", (B,), torch.int64, dev)
    if not (0 <= n_uniform <= S):
        raise ValueError("n_uniform must be in [0, sample_size]")
    n_draws = sampler_draws_count(sampler, B, S, n_uniform)
    if exp_draws is not None:
        if n_draws == 0:
            raise ValueError("exp_draws needs a drawing sampler (COMPOSITE, TRAJECTORY, DECISION_BOUNDARY)")
        exp_draws = _need(exp_draws.reshape(-1), "exp_draws", (n_draws,), torch.float32, dev)
    if sampler == L.FIODE_SAMPLER_GIVEN:
        if h is None:
            raise ValueError("sampler GIVEN needs h")
        h = _need(h, "h", (N, C), torch.float32, dev)
    if sampler == L.FIODE_SAMPLER_TRAJECTORY and n_uniform < S:
        if h is None:
            raise ValueError("sampler TRAJECTORY needs the trajectory rows h [B, S - n_uniform, C]")
        h = _need(h, "h", (B, S - n_uniform, C), torch.float32, dev)
    if dropout_mode == L.FIODE_DROPOUT_GIVEN:
        if masks is None:
            raise ValueError("dropout GIVEN needs masks")
        masks = _need(masks, "masks", (4, N, M), torch.uint8, dev)
    if offset_dev is not None:
        offset_dev = _need(offset_dev, "offset_dev", (1,), torch.int64, dev)
    ws_w, cw = _weights_c(weights, dev)
    if out is None:
        out = {}
    grads = out.get("grads")
    if grads is None:
        grads = {k: torch.empty(WEIGHT_SHAPES[k], dtype=torch.float32, device=dev) for k in WEIGHT_KEYS}
        grads["x_feat"] = torch.empty((B, X), dtype=torch.float32, device=dev)
        out["grads"] = grads
    scalars = out.get("scalars")
    if scalars is None:
        scalars = torch.empty(8, dtype=torch.float32, device=dev)
        out["scalars"] = scalars
    dbg = {}
    if debug:
        dbg = dict(h=torch.empty((N, C), device=dev), V=torch.empty(N, device=dev), Vdot=torch.empty(N, device=dev),
                   f=torch.empty((N, C), device=dev), f_log=torch.empty((N, C), device=dev),
                   qp_lower=torch.empty((N, C), device=dev), qp_nominal=torch.empty((2, N, C), device=dev),
                   g_ftilde=torch.empty((N, C), device=dev),
                   keep_words=torch.empty((4, N, 4), dtype=torch.int32, device=dev))
        if n_draws:
            dbg["exp_draws"] = torch.empty(n_draws, dtype=torch.float32, device=dev)
    if kappa_dev is not None:
        kappa_dev = _need(kappa_dev.reshape(1), "kappa_dev", (1,), torch.float32, dev)
    cfg = L.LyapConfig(B, S, int(n_uniform), int(sampler), int(dropout_mode), float(kappa),
                       int(seed) & (2**64 - 1), int(offset) & (2**64 - 1))
    dc = dyn.to_c()
    ev_arr, n_ev = None, 0
    if events is not None:
        if len(events) < len(L.LYAP_KERNELS) + 1:
            raise ValueError("need len(LYAP_KERNELS)+1 events")
        st = torch.cuda.current_stream(dev)
        for e in events:          # torch creates the hipEvent lazily on first record
            if e.cuda_event == 0:
                e.record(st)
        ev_arr = (ct.c_void_p * len(events))(*[e.cuda_event for e in events])
        n_ev = len(events)
    io = L.LyapIO(x_feat.data_ptr(), y.data_ptr(), _ptr(h), _ptr(masks), scalars.data_ptr(),
                  _ptr(dbg.get("h")), _ptr(dbg.get("V")), _ptr(dbg.get("Vdot")), _ptr(dbg.get("f")),
                  _ptr(dbg.get("f_log")), _ptr(dbg.get("qp_lower")), _ptr(dbg.get("qp_nominal")),
                  _ptr(dbg.get("g_ftilde")), ct.cast(ev_arr, ct.c_void_p) if ev_arr is not None else None, n_ev,
                  _ptr(offset_dev), _ptr(exp_draws), _ptr(dbg.get("exp_draws")), _ptr(dbg.get("keep_words")),
                  _ptr(kappa_dev))
    cg = L.LyapGrads(*[grads[k].data_ptr() for k in WEIGHT_KEYS + ("x_feat",)])
    lib = L.lib()
    nbytes = lib.fiode_lyap_workspace_bytes(ct.byref(cfg), ct.byref(dc))
    ws = _Workspace.get(dev, nbytes, "lyap")
    rc = lib.fiode_lyap_step(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), ct.byref(io), ct.byref(cg),
                             ct.c_void_p(ws.data_ptr()), ct.c_size_t(ws.numel()))
    L.check(rc, "fiode_lyap_step")
    del ws_w
    return scalars, grads, dbg


def qp_forward(lower: torch.Tensor, nominal: torch.Tensor, max_iter: int = 30, tol: float = 1e-4):
    """FastBarrierProjectionNoUpper forward (batch-global exit).  Returns (v, mu[N], exit_iter[1])."""
    dev = nominal.device
    n = nominal.shape[0]
    lower = _need(lower, "lower", (n, C), torch.float32, dev)
    nominal = _need(nominal, "nominal", (n, C), torch.float32, dev)
    v = torch.empty_like(nominal)
    mu = torch.empty(n, dtype=torch.float32, device=dev)
    it = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = _Workspace.get(dev, 256, "qp")
    rc = L.lib().fiode_qp_forward(_stream(dev), n, C, lower.data_ptr(), nominal.data_ptr(), int(max_iter),
                                  float(tol), v.data_ptr(), mu.data_ptr(), it.data_ptr(), ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_qp_forward")
    return v, mu, it


def qp_backward(g, v, mu, lower, nominal):
    dev = v.device
    n = v.shape[0]
    g = _need(g, "g", (n, C), torch.float32, dev)
    v = _need(v, "v", (n, C), torch.float32, dev)
    mu = _need(mu.reshape(-1), "mu", (n,), torch.float32, dev)
    nominal = _need(nominal, "nominal", (n, C), torch.float32, dev)
    lower = _need(lower, "lower", (n, C), torch.float32, dev)
    gl = torch.empty_like(v)
    gn = torch.empty_like(v)
    rc = L.lib().fiode_qp_backward(_stream(dev), n, C, g.data_ptr(), v.data_ptr(), mu.data_ptr(), lower.data_ptr(),
                                   nominal.data_ptr(), gl.data_ptr(), gn.data_ptr())
    L.check(rc, "fiode_qp_backward")
    return gl, gn


def dyn_eval(h: torch.Tensor, x_feat: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg,
             rows_per_image: int = 1):
    """eval_dot in eval mode: f[N][C] for h[N][C]; row r uses x_feat[r // rows_per_image]."""
    dev = h.device
    n = h.shape[0]
    B = x_feat.shape[0]
    if B * rows_per_image != n:
        raise ValueError("h rows must equal batch * rows_per_image")
    h = _need(h, "h", (n, C), torch.float32, dev)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    ws_w, cw = _weights_c(weights, dev)
    f = torch.empty_like(h)
    it = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = L.lib()
    ws = _Workspace.get(dev, lib.fiode_dyn_eval_workspace_bytes(n), "dyn")
    dc = dyn.to_c()
    rc = lib.fiode_dyn_eval(_stream(dev), ct.byref(dc), ct.byref(cw), B, int(rows_per_image), x_feat.data_ptr(),
                            h.data_ptr(), f.data_ptr(), it.data_ptr(), ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_dyn_eval")
    return f, it


def odeint_dyn(x_feat: torch.Tensor, h0: torch.Tensor, times: torch.Tensor, weights: Dict[str, torch.Tensor],
               dyn: DynCfg, method: str = "dopri5", rtol: float = 1e-3, atol: float = 1e-3,
               step_size: Optional[float] = None, max_steps: int = 100000):
    """fiode_odeint: solve dh/dt = eval_dot(h, x_feat) (eval mode) from h0 over ``times``.
    Returns (solution [T,B,C], stats int32[8], dstats float64[4]) -- all on the device."""
    dev = h0.device
    B = h0.shape[0]
    if B > L.FIODE_ODEINT_MAX_BATCH:
        raise ValueError(f"batch {B} > FIODE_ODEINT_MAX_BATCH")
    h0 = _need(h0, "h0", (B, C), torch.float32, dev)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    T = times.shape[0]
    times = _need(times.reshape(-1), "times", (T,), torch.float64, dev)
    if method == "rk4":
        if step_size is None or not step_size > 0:
            raise ValueError("rk4 needs options.step_size > 0")
        m = L.FIODE_ODE_RK4
    elif method == "dopri5":
        m = L.FIODE_ODE_DOPRI5
    else:
        raise NotImplementedError(f"method {method!r}: the HIP stepper implements 'rk4' and 'dopri5'")
    ws_w, cw = _weights_c(weights, dev)
    sol = torch.empty((T, B, C), dtype=torch.float32, device=dev)
    stats = torch.zeros(8, dtype=torch.int32, device=dev)
    dstats = torch.zeros(4, dtype=torch.float64, device=dev)
    cfg = L.OdeConfig(m, B, T, int(max_steps), float(rtol), float(atol), float(step_size or 0.0))
    lib = L.lib()
    ws = _Workspace.get(dev, lib.fiode_odeint_workspace_bytes(B), "ode")
    dc = dyn.to_c()
    rc = lib.fiode_odeint(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), x_feat.data_ptr(), h0.data_ptr(),
                          times.data_ptr(), sol.data_ptr(), stats.data_ptr(), dstats.data_ptr(), ws.data_ptr(),
                          ws.numel())
    L.check(rc, "fiode_odeint")
    del ws_w
    return sol, stats, dstats


def odetrain_config(B: int, t0: float, t1: float, step_size: float, dropout_mode: int, seed: int = 0,
                    offset: int = 0, method: str = "rk4", rtol: float = 1e-3, atol: float = 1e-3,
                    max_attempts: int = 64) -> L.OdeTrainConfig:
    """The differentiable train_ode solve: method 'rk4' (step_size) or 'dopri5' (rtol, atol; at most
    max_attempts adaptive step attempts -- the eval capacity is 2 + 6 max_attempts)."""
    m = {"rk4": L.FIODE_ODE_RK4, "dopri5": L.FIODE_ODE_DOPRI5}[method]
    return L.OdeTrainConfig(int(B), int(dropout_mode), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1),
                            float(t0), float(t1), float(step_size), m, int(max_attempts), float(rtol), float(atol))


ODETRAIN_ATTEMPT_BUDGET = 4 << 30       # bytes of dopri5 workspace the default attempt capacity may use


def odetrain_default_attempts(B: int, budget_bytes: int = ODETRAIN_ATTEMPT_BUDGET) -> int:
    """Attempt capacity of the differentiable dopri5 solve when the caller sets none: as many
    attempts as ``budget_bytes`` of workspace hold (each attempt saves 6 evals' stage inputs,
    activations and QP state for the backward), capped at FIODE_ODETRAIN_MAX_ATTEMPTS.  torchdiffeq's
    loop is uncapped (max_num_steps 2**31 - 1); exhausting the capacity is status 2 (stated
    deviation).  At B = 128 this is the maximum, 1,024 attempts (~1.9 GB); at
    B = 1,024, ~280 (configs[4]'s solve takes ~35)."""
    lib = L.lib()
    w = [lib.fiode_odetrain_workspace_bytes(ct.byref(odetrain_config(B, 0.0, 1.0, 0.0, L.FIODE_DROPOUT_OFF,
                                                                      method="dopri5", max_attempts=a)))
         for a in (1, 2)]
    per = max(1, w[1] - w[0])
    return int(max(64, min(L.FIODE_ODETRAIN_MAX_ATTEMPTS, (budget_bytes - w[0]) // per + 1)))


def odetrain_evals(cfg: L.OdeTrainConfig) -> int:
    E = L.lib().fiode_odetrain_evals(ct.byref(cfg))
    if E < 0:
        raise ValueError("odetrain: invalid solve (rk4: t1 > t0, step_size > 0, <= 1024 steps; dopri5: rtol, atol > 0, "
                         "1 <= max_attempts <= 1024)")
    return E




def odetrain_forward(x_feat: torch.Tensor, h0: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg,
                     cfg: L.OdeTrainConfig, masks: Optional[torch.Tensor] = None,
                     offset_dev: Optional[torch.Tensor] = None):
    """fiode_odetrain_forward: y(t1) of the train-mode RK4 solve.  Returns (y [B,C], stats int32[8],
    workspace) -- the workspace carries the saved activations to ``odetrain_backward``."""
    dev = h0.device
    B = int(cfg.batch)
    if B > L.FIODE_ODE_MAX_BATCH:
        raise ValueError(f"batch {B} > FIODE_ODE_MAX_BATCH")
    h0 = _need(h0, "h0", (B, C), torch.float32, dev)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    E = odetrain_evals(cfg)
    if cfg.dropout_mode == L.FIODE_DROPOUT_GIVEN:
        if masks is None:
            raise ValueError("dropout GIVEN needs masks [E,2,B,M]")
        masks = _need(masks, "masks", (E, 2, B, M), torch.uint8, dev)
    if offset_dev is not None:
        offset_dev = _need(offset_dev, "offset_dev", (1,), torch.int64, dev)
    lib = L.lib()
    ws = torch.empty(lib.fiode_odetrain_workspace_bytes(ct.byref(cfg)), dtype=torch.uint8, device=dev)
    ws_w, cw = _weights_c(weights, dev)
    y = torch.empty((B, C), dtype=torch.float32, device=dev)
    # k_ot_masks zeroes the stats words itself (a zero fill here ran on the chain ahead of the solve)
    stats = torch.empty(8, dtype=torch.int32, device=dev)
    dc = dyn.to_c()
    rc = lib.fiode_odetrain_forward(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), x_feat.data_ptr(),
                                    h0.data_ptr(), _ptr(masks), _ptr(offset_dev), y.data_ptr(), stats.data_ptr(),
                                    ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_odetrain_forward")
    del ws_w
    return y, stats, ws


def odetrain_saved(ws: torch.Tensor, cfg: L.OdeTrainConfig) -> Dict[str, torch.Tensor]:
    """Views of the forward's saved arrays in an odetrain workspace (for checkers)."""
    B, E = int(cfg.batch), odetrain_evals(cfg)
    off = (ct.c_int64 * L.FIODE_ODETRAIN_NSAVED)()
    L.check(L.lib().fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(off, ct.c_void_p)),
            "fiode_odetrain_saved_offsets")
    f = lambda i, n: ws[off[i]:off[i] + 4 * n].view(torch.float32)
    R = B * E
    out = dict(h=f(0, R * C).view(B, E, C), ftilde=f(1, R * C).view(B, E, C), v=f(2, R * C).view(B, E, C),
               mu=f(3, R).view(B, E), nominal=f(4, R * C).view(B, E, C), a1=f(5, R * M).view(B, E, M),
               a2=f(6, R * M).view(B, E, M), gft=f(7, R * C).view(B, E, C), lower=f(8, R * C).view(B, E, C),
               status=ws[off[12]:off[12] + 4].view(torch.int32),
               keep_words=ws[off[13]:off[13] + E * 2 * B * 16].view(torch.int32).view(E, 2, B, 4))
    if cfg.method == L.FIODE_ODE_DOPRI5:
        A = int(cfg.max_attempts)
        out["ys"] = f(9, A * B * C).view(A, B, C)
        out["attempts"] = ws[off[10]:off[10] + 8 * 8 * A].view(torch.float64).view(A, 8)
        out["init"] = ws[off[11]:off[11] + 8 * 16].view(torch.float64)
    return out


def odetrain_status_word(ws: torch.Tensor, cfg: L.OdeTrainConfig) -> torch.Tensor:
    """int32 [1] view of the solve's status word in an odetrain workspace (saved entry 12: dopri5
    forward + backward status, 0 ok; rk4 keeps it 0 -- its forward status is stats[3])."""
    off = (ct.c_int64 * L.FIODE_ODETRAIN_NSAVED)()
    L.check(L.lib().fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(off, ct.c_void_p)),
            "fiode_odetrain_saved_offsets")
    return ws[off[12]:off[12] + 4].view(torch.int32)


def odetrain_backward(g_y: torch.Tensor, x_feat: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg,
                      cfg: L.OdeTrainConfig, ws: torch.Tensor, debug: bool = False):
    """fiode_odetrain_backward: dL/d(weights, x_feat) from dL/dy(t1).  Returns (grads, dbg_gft)."""
    dev = g_y.device
    B = int(cfg.batch)
    g_y = _need(g_y.float(), "g_y", (B, C), torch.float32, dev)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    E = odetrain_evals(cfg)
    ws_w, cw = _weights_c(weights, dev)
    grads = {k: torch.empty(WEIGHT_SHAPES[k], dtype=torch.float32, device=dev) for k in WEIGHT_KEYS}
    grads["x_feat"] = torch.empty((B, X), dtype=torch.float32, device=dev)
    cg = L.LyapGrads(*[grads[k].data_ptr() for k in WEIGHT_KEYS + ("x_feat",)])
    dbg = torch.empty((B, E, C), dtype=torch.float32, device=dev) if debug else None
    dc = dyn.to_c()
    rc = L.lib().fiode_odetrain_backward(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), x_feat.data_ptr(),
                                         g_y.data_ptr(), ct.byref(cg), _ptr(dbg), ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_odetrain_backward")
    del ws_w
    return grads, dbg


def odetrain_backward_x(g_y: torch.Tensor, x_feat: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg,
                        cfg: L.OdeTrainConfig, ws: torch.Tensor, gx_add: Optional[torch.Tensor] = None,
                        gx_add_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fiode_odetrain_backward_x: the adjoint sweep and dL/dx_feat [B, X] (+ gx_add * gx_add_scale,
    a device scalar).  ``odetrain_backward_weights`` on the same workspace completes the gradients."""
    dev = g_y.device
    B = int(cfg.batch)
    g_y = _need(g_y.float(), "g_y", (B, C), torch.float32, dev)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    if gx_add is not None:
        gx_add = _need(gx_add, "gx_add", (B, X), torch.float32, dev)
        gx_add_scale = _need(gx_add_scale.reshape(1), "gx_add_scale", (1,), torch.float32, dev)
    ws_w, cw = _weights_c(weights, dev)
    gx = torch.empty((B, X), dtype=torch.float32, device=dev)
    dc = dyn.to_c()
    rc = L.lib().fiode_odetrain_backward_x(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), x_feat.data_ptr(),
                                           g_y.data_ptr(), gx.data_ptr(), _ptr(gx_add),
                                           _ptr(gx_add_scale if gx_add is not None else None), None, ws.data_ptr(),
                                           ws.numel())
    L.check(rc, "fiode_odetrain_backward_x")
    del ws_w
    return gx


def odetrain_backward_weights(x_feat: torch.Tensor, weights: Dict[str, torch.Tensor], dyn: DynCfg,
                              cfg: L.OdeTrainConfig, ws: torch.Tensor) -> Dict[str, torch.Tensor]:
    """fiode_odetrain_backward_weights: the eight weight gradients (after odetrain_backward_x)."""
    dev = x_feat.device
    B = int(cfg.batch)
    x_feat = _need(x_feat, "x_feat", (B, X), torch.float32, dev)
    ws_w, cw = _weights_c(weights, dev)
    grads = {k: torch.empty(WEIGHT_SHAPES[k], dtype=torch.float32, device=dev) for k in WEIGHT_KEYS}
    cg = L.LyapGrads(*([grads[k].data_ptr() for k in WEIGHT_KEYS] + [None]))
    dc = dyn.to_c()
    rc = L.lib().fiode_odetrain_backward_weights(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw),
                                                 x_feat.data_ptr(), ct.byref(cg), ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_odetrain_backward_weights")
    del ws_w
    return grads


def certify_grid(T: int = 40, n: int = C, device="cuda") -> torch.Tensor:
    """grid_label_0 of sample_decision_boundary(n, T) as uint8 counts [G][n] (eta = v/T)."""
    lib = L.lib()
    G = lib.fiode_certify_grid_rows(n, T)
    if G < 0:
        raise ValueError(f"unsupported grid n={n} T={T}")
    dev = torch.device(device)
    grid = torch.empty((max(G, 1), n), dtype=torch.uint8, device=dev)
    L.check(lib.fiode_certify_grid(_stream(dev), n, T, grid.data_ptr()), "fiode_certify_grid")
    return grid[:G]


def certify_image(x_feat: torch.Tensor, label: int, grid: torch.Tensor, weights: Dict[str, torch.Tensor],
                  dyn: DynCfg, T: int = 40, batches: int = 10, eps: float = 0.141, min_std: float = 0.225):
    """One image of certify_lipschitz.py:104-143: returns (out [nb][2] = per-batch max violation and
    max violation_larger_T, exit_iters [nb]) on the device."""
    dev = grid.device
    G = grid.shape[0]
    x_feat = _need(x_feat.reshape(-1), "x_feat", (X,), torch.float32, dev)
    grid = _need(grid, "grid", (G, C), torch.uint8, dev)
    nb = batches + (1 if G % batches else 0)
    out = torch.empty((nb, 2), dtype=torch.float32, device=dev)
    it = torch.empty(nb, dtype=torch.int32, device=dev)
    ws_w, cw = _weights_c(weights, dev)
    lib = L.lib()
    ws = _Workspace.get(dev, lib.fiode_certify_workspace_bytes(G, batches), "cert")
    cfg = L.CertifyConfig(C, int(T), int(batches), int(label), float(eps), float(min_std))
    dc = dyn.to_c()
    rc = lib.fiode_certify(_stream(dev), ct.byref(cfg), ct.byref(dc), ct.byref(cw), x_feat.data_ptr(), grid.data_ptr(),
                           G, out.data_ptr(), it.data_ptr(), ws.data_ptr(), ws.numel())
    L.check(rc, "fiode_certify")
    del ws_w
    return out, it


def batched_inverse(M: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(..., n, n) -> inverse, n <= 128, float32 or complex64 (fiode_batched_inverse).
    Valid for matrices with positive-definite Hermitian part (the Cayley I + A)."""
    if M.device.type != "cuda":
        raise ValueError(f"batched_inverse: must be on a ROCm device; got {M.device}")
    if M.dtype not in (torch.float32, torch.complex64):
        raise TypeError(f"batched_inverse: dtype {M.dtype} (float32 / complex64 only)")
    n = M.shape[-1]
    if M.dim() < 2 or M.shape[-2] != n or n > L.FIODE_INV_MAX_N:
        raise ValueError(f"batched_inverse: shape {tuple(M.shape)} (square, n <= {L.FIODE_INV_MAX_N})")
    M = M.contiguous()
    if out is None:
        out = torch.empty_like(M)
    batch = M.numel() // (n * n)
    dt = L.FIODE_DTYPE_F32 if M.dtype == torch.float32 else L.FIODE_DTYPE_C64
    L.check(L.lib().fiode_batched_inverse(_stream(M.device), dt, batch, n, M.data_ptr(), n * n, out.data_ptr(),
                                          n * n), "fiode_batched_inverse")
    return out


def block_inverse(M: torch.Tensor, out: Optional[torch.Tensor] = None,
                  skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(n, n) or (b, n, n) float32 -> inverse by 64-wide panel block Gauss-Jordan on the device
    (fiode_block_inverse[_batched]: one launch sequence for the whole batch).  Valid for matrices
    with positive-definite symmetric part.  ``skip``: device int32 scalar; nonzero = the launches
    return at once and ``out`` is left as it is (fiode_block_inverse_cond)."""
    if (M.device.type != "cuda" or M.dtype != torch.float32 or M.dim() not in (2, 3)
            or M.shape[-1] != M.shape[-2]):
        raise ValueError(f"block_inverse: square float32 ROCm matrix expected, got {tuple(M.shape)} {M.dtype} "
                         f"on {M.device}")
    n = int(M.shape[-1])
    b = 1 if M.dim() == 2 else int(M.shape[0])
    M = M.contiguous()
    if out is None:
        out = torch.empty_like(M)
    lib = L.lib()
    nb = lib.fiode_block_inverse_workspace_bytes(n) * b
    ws = _Workspace.get(M.device, nb, f"blockinv{torch.cuda.current_stream(M.device).cuda_stream}")
    if skip is not None:
        skip = _need(skip.reshape(1), "skip", (1,), torch.int32, M.device)
    L.check(lib.fiode_block_inverse_cond(_stream(M.device), b, n, M.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                         ws.numel(), _ptr(skip)), "fiode_block_inverse_cond")
    return out


def sconv_rfft2(x: Optional[torch.Tensor], n: int, C: int, B: int, downsample: bool = False,
                gy: Optional[torch.Tensor] = None, code: Optional[torch.Tensor] = None,
                nchw: bool = False) -> torch.Tensor:
    """fiode_sconv_rfft2: spatial-major x [n][n][C][B] (downsample: [2n][2n][C/4][B]) -> complex64
    [n (n/2+1), C, B].  With gy/code: the transform of GroupSort's backward of gy [n][n][C][B]
    (nchw: gy [B][C][n][n] and codes [B][C/2][n][n], as sconv_irfft2(nchw=True) wrote them)."""
    src = gy if gy is not None else x
    dev = src.device
    if nchw and gy is None:
        raise ValueError("sconv_rfft2: nchw only for the GroupSort-backward input (gy)")
    if gy is not None:
        gy = _need(gy, "gy", (B, C, n, n) if nchw else (n, n, C, B), torch.float32, dev)
        code = _need(code, "code", (B, C // 2, n, n) if nchw else (n, n, C // 2, B), torch.uint8, dev)
    else:
        shape = (2 * n, 2 * n, C // 4, B) if downsample else (n, n, C, B)
        x = _need(x, "x", shape, torch.float32, dev)
    X = torch.empty((n * (n // 2 + 1), C, B), dtype=torch.complex64, device=dev)
    cfg = L.SconvConfig(n, C, B, int(bool(downsample)), int(bool(nchw)))
    L.check(L.lib().fiode_sconv_rfft2(_stream(dev), ct.byref(cfg), _ptr(x), _ptr(gy), _ptr(code), X.data_ptr()),
            "fiode_sconv_rfft2")
    return X


def sconv_rfft2_nchw(x: torch.Tensor, mu: torch.Tensor, sd: Optional[torch.Tensor], n: int) -> torch.Tensor:
    """fiode_sconv_rfft2_nchw: X = rfft2((x - mu) / sd) of an NCHW input x [B][C][n][n] -> complex64
    [n (n/2+1), C, B] (the first conv with the backbone's Normalize fused)."""
    dev = x.device
    B, C = x.shape[0], x.shape[1]
    x = _need(x, "x", (B, C, n, n), torch.float32, dev)
    mu = _need(mu.detach().reshape(-1), "mu", (C,), torch.float32, dev)
    if sd is not None:
        sd = _need(sd.detach().reshape(-1), "sd", (C,), torch.float32, dev)
    X = torch.empty((n * (n // 2 + 1), C, B), dtype=torch.complex64, device=dev)
    cfg = L.SconvConfig(n, C, B, 0, 0)
    L.check(L.lib().fiode_sconv_rfft2_nchw(_stream(dev), ct.byref(cfg), x.data_ptr(), mu.data_ptr(), _ptr(sd),
                                           X.data_ptr()), "fiode_sconv_rfft2_nchw")
    return X


def sconv_irfft2(Y: torch.Tensor, n: int, C: int, B: int, bias: Optional[torch.Tensor] = None,
                 groupsort: bool = False, downsample: bool = False, nchw: bool = False):
    """fiode_sconv_irfft2: complex64 [n (n/2+1), C, B] -> y [n][n][C][B] (+ bias; GroupSort with its
    comparison codes [n][n][C/2][B]; or downsample: scattered to [2n][2n][C/4][B]; nchw: y
    [B][C][n][n], codes [B][C/2][n][n])."""
    dev = Y.device
    Y = _need(Y, "Y", (n * (n // 2 + 1), C, B), torch.complex64, dev)
    if bias is not None:
        bias = _need(bias.detach(), "bias", (C,), torch.float32, dev)
    if nchw and downsample:
        raise ValueError("sconv_irfft2: nchw and downsample together")
    shape = (2 * n, 2 * n, C // 4, B) if downsample else ((B, C, n, n) if nchw else (n, n, C, B))
    y = torch.empty(shape, dtype=torch.float32, device=dev)
    code = (torch.empty((B, C // 2, n, n) if nchw else (n, n, C // 2, B), dtype=torch.uint8, device=dev)
            if groupsort else None)
    cfg = L.SconvConfig(n, C, B, int(bool(downsample)), int(bool(nchw)))
    L.check(L.lib().fiode_sconv_irfft2(_stream(dev), ct.byref(cfg), Y.data_ptr(), _ptr(bias), int(bool(groupsort)),
                                       y.data_ptr(), _ptr(code)), "fiode_sconv_irfft2")
    return y, code


def sconv_irfft2_qx(Q: torch.Tensor, X: torch.Tensor, n: int, B: int, bias: Optional[torch.Tensor] = None,
                    groupsort: bool = False, nchw: bool = False):
    """fiode_sconv_irfft2_qx: sconv_irfft2(Q @ X) with the per-frequency product formed in the
    transform's loads (few input channels: Q [n (n/2+1), C, K], X [n (n/2+1), K, B], K <= 4)."""
    dev = X.device
    nf = n * (n // 2 + 1)
    if Q.dim() != 3 or Q.shape[0] != nf:
        raise ValueError(f"sconv_irfft2_qx: Q {tuple(Q.shape)} is not [{nf}, C, K]")
    C, K = Q.shape[1], Q.shape[2]
    Q = _need(Q.detach(), "Q", (nf, C, K), torch.complex64, dev)
    X = _need(X.detach(), "X", (nf, K, B), torch.complex64, dev)
    if bias is not None:
        bias = _need(bias.detach(), "bias", (C,), torch.float32, dev)
    y = torch.empty((B, C, n, n) if nchw else (n, n, C, B), dtype=torch.float32, device=dev)
    code = (torch.empty((B, C // 2, n, n) if nchw else (n, n, C // 2, B), dtype=torch.uint8, device=dev)
            if groupsort else None)
    cfg = L.SconvConfig(n, C, B, 0, int(bool(nchw)))
    L.check(L.lib().fiode_sconv_irfft2_qx(_stream(dev), ct.byref(cfg), Q.data_ptr(), X.data_ptr(), K, _ptr(bias),
                                          int(bool(groupsort)), y.data_ptr(), _ptr(code)), "fiode_sconv_irfft2_qx")
    return y, code


def cgemm(A: torch.Tensor, B: torch.Tensor, conj_trans_a: bool = False, conj_trans_b: bool = False,
          scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fiode_cgemm: batched complex64 C[f] = scale[f] opA(A[f]) @ opB(B[f]); A [F, M, K] ([F, K, M]
    with conj_trans_a: A^H), B [F, K, N] ([F, N, K] with conj_trans_b: B^H), scale [F] float32."""
    dev = B.device
    if A.dim() != 3 or B.dim() != 3 or A.dtype != torch.complex64 or B.dtype != torch.complex64:
        raise ValueError(f"cgemm: complex64 [F, ., .] operands, got {tuple(A.shape)} {A.dtype}, "
                         f"{tuple(B.shape)} {B.dtype}")
    if conj_trans_a and conj_trans_b:
        raise ValueError("cgemm: conj_trans_a and conj_trans_b together are not supported")
    F = B.shape[0]
    K, N = (B.shape[2], B.shape[1]) if conj_trans_b else (B.shape[1], B.shape[2])
    M, ka = (A.shape[2], A.shape[1]) if conj_trans_a else (A.shape[1], A.shape[2])
    if A.shape[0] != F or ka != K or A.device != dev:
        raise ValueError(f"cgemm: A {tuple(A.shape)} does not match B {tuple(B.shape)}")
    if scale is not None:
        scale = _need(scale.detach().reshape(-1), "scale", (F,), torch.float32, dev)
    A = A.contiguous()
    B = B.contiguous()
    C = torch.empty((F, M, N), dtype=torch.complex64, device=dev)
    L.check(L.lib().fiode_cgemm(_stream(dev), F, M, N, K, int(bool(conj_trans_a)), int(bool(conj_trans_b)),
                                _ptr(scale), A.data_ptr(), B.data_ptr(), C.data_ptr()), "fiode_cgemm")
    return C


def _mat_layout(X: torch.Tensor):
    """(trans, ld) of a 2-D (or the last two dims of a batched) float32 view X [R, Cn] over row-major
    memory: X itself row-major (unit inner stride) -> (0, row stride); X the transposed view of a
    row-major matrix -> (1, its row stride); else None (the caller copies)."""
    R, Cn = X.shape[-2], X.shape[-1]
    s0, s1 = X.stride(-2), X.stride(-1)
    if (s1 == 1 or Cn == 1) and (s0 >= Cn or R == 1):
        return 0, max(s0 if R > 1 else Cn, Cn, 1)
    if (s0 == 1 or R == 1) and (s1 >= R or Cn == 1):
        return 1, max(s1 if Cn > 1 else R, R, 1)
    return None


# GEMM routing.  ops.mm call sites named here take the library GEMM (torch.matmul / addmm: hipBLASLt)
# instead of fiode_gemm: on the step's shapes fiode_gemm's 64 x 64 tiles run 63-65 TF/s where the
# library's tuned tiles (224 x 32, 32 x 32 x 128 ...) run 83-90 on the 512-map products and twice
# as fast on the head's skinny ones (profiles/r06/gemm_probe_prefetch.log), and the same-box step
# A/B with a copy-free library route measured 1.2404 (library at all three sites) vs 1.2905 ms
# (fiode_gemm everywhere); each site alone: dense_fwd -14, dense_bwd -10, head -24 us
# (profiles/r06/ab_gemm_sites.json).  fiode_gemm stays the C-ABI product (tested bit-for-bit
# against itself and to fp32 tolerance against the library) for any site a faster tile wins back.
# MM_LIBRARY (tools/ab_step.py `lib_gemm`) routes every call to the library.
MM_LIBRARY = False
MM_LIBRARY_SITES: set = {"dense_fwd", "dense_bwd", "head"}
# the dense maps' backward pair (A, P2) in one fiode_gemm_pair launch (tools/ab_step.py `no_pair`: two launches)
MM_PAIR = True


def _gemm_ws(dev: torch.device, nbytes: int) -> torch.Tensor:
    # one split-K workspace per stream (its counter words are zero on entry and left zero by every
    # call; calls on one stream are ordered, calls on two streams never share a workspace)
    return _Workspace.get(dev, nbytes, f"gemm{torch.cuda.current_stream(dev).cuda_stream}", zero=True)


def _gemm_operands(A: torch.Tensor, B: torch.Tensor, alpha: float, beta: float, bias, out, split_k: int,
                   max_workgroups: int):
    """The fiode_gemm_desc of out = alpha A @ B + beta out + bias, with the operands as the kernel reads
    them (a view it cannot read in place copied) and the output allocated when not given."""
    dev = B.device
    if A.dtype != torch.float32 or B.dtype != torch.float32 or A.device != dev or dev.type != "cuda":
        raise ValueError(f"mm: float32 ROCm operands, got {A.dtype} on {A.device}, {B.dtype} on {B.device}")
    if A.dim() not in (2, 3) or B.dim() not in (2, 3) or A.shape[-1] != B.shape[-2]:
        raise ValueError(f"mm: shapes {tuple(A.shape)} @ {tuple(B.shape)}")
    batch = max(A.shape[0] if A.dim() == 3 else 1, B.shape[0] if B.dim() == 3 else 1)
    for X in (A, B):
        if X.dim() == 3 and X.shape[0] != batch:
            raise ValueError(f"mm: batch sizes {tuple(A.shape)} / {tuple(B.shape)}")
    M, K, N = A.shape[-2], A.shape[-1], B.shape[-1]
    la = _mat_layout(A)
    if la is None:
        A = A.contiguous()
        la = _mat_layout(A)
    lb = _mat_layout(B)
    if lb is None:
        B = B.contiguous()
        lb = _mat_layout(B)
    oshape = (batch, M, N) if (A.dim() == 3 or B.dim() == 3) else (M, N)
    if out is None:
        if beta != 0.0:
            raise ValueError("mm: beta needs out")
        out = torch.empty(oshape, dtype=torch.float32, device=dev)
    elif (tuple(out.shape) != oshape or out.dtype != torch.float32 or out.device != dev or
          (out.dim() == 2 and not (out.stride(1) == 1 and out.stride(0) >= N)) or
          (out.dim() == 3 and not out.is_contiguous())):
        raise ValueError(f"mm: out must be a float32 {oshape} tensor on {dev} with unit column stride "
                         "(contiguous when batched)")
    ldc = out.stride(-2) if out.dim() == 2 else N
    if bias is not None:
        bias = _need(bias.detach(), "bias", (N,), torch.float32, dev)
    d = L.GemmDesc(batch, M, N, K, la[0], lb[0], la[1], lb[1], ldc,
                   A.stride(0) if A.dim() == 3 else 0, B.stride(0) if B.dim() == 3 else 0, M * N,
                   float(alpha), float(beta), int(split_k), int(max_workgroups))
    return d, A, B, bias, out


def mm(A: torch.Tensor, B: torch.Tensor, *, alpha: float = 1.0, beta: float = 0.0,
       bias: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, split_k: int = 0,
       max_workgroups: int = 0, site: str = "") -> torch.Tensor:
    """fiode_gemm: out = alpha A @ B + beta out + bias, float32, A [(b,) M, K], B [(b,) K, N] (a 2-D
    operand is shared by every batch entry), bias [N].  Either operand may be a transposed view of
    row-major memory (``W.t()``, ``X.mT``, a column slice): the kernel reads it in place.  The hand-
    written replacement of torch.matmul / addmm on the Cayley layers' products (gemm.hip).
    ``max_workgroups``: a capped, persistent grid (a narrow launch beside other work; 0 = none)."""
    dev = B.device
    if MM_LIBRARY or site in MM_LIBRARY_SITES:   # the library GEMM (routing note above)
        if out is None and alpha == 1.0 and beta == 0.0:        # round 5's calls: no copy
            if bias is not None and A.dim() == 2 and B.dim() == 2:
                return torch.addmm(bias, A, B)
            r = torch.matmul(A, B)
            return (r + bias if bias is not None else r).contiguous()
        d, A, B, bias, out = _gemm_operands(A, B, alpha, beta, bias, out, split_k, max_workgroups)
        r = torch.matmul(A, B)
        r = r * alpha if alpha != 1.0 else r
        if bias is not None:
            r = r + bias
        if beta != 0.0:
            r = r + beta * out
        out.copy_(r)
        return out
    d, A, B, bias, out = _gemm_operands(A, B, alpha, beta, bias, out, split_k, max_workgroups)
    lib = L.lib()
    nb = lib.fiode_gemm_workspace_bytes(ct.byref(d))
    ws = _gemm_ws(dev, nb) if nb else None
    L.check(lib.fiode_gemm(_stream(dev), ct.byref(d), A.data_ptr(), B.data_ptr(), _ptr(bias), out.data_ptr(),
                           _ptr(ws), ws.numel() if ws is not None else 0), "fiode_gemm")
    return out


def mm_pair(A0: torch.Tensor, B0: torch.Tensor, A1: torch.Tensor, B1: torch.Tensor, site: str = ""):
    """fiode_gemm_pair: (A0 @ B0, A1 @ B1) -- two independent products in one launch, each the same
    bits as ``mm`` computes it."""
    if MM_LIBRARY or not MM_PAIR or site in MM_LIBRARY_SITES:
        return mm(A0, B0, site=site), mm(A1, B1, site=site)
    dev = B0.device
    d0, A0, B0, _, C0 = _gemm_operands(A0, B0, 1.0, 0.0, None, None, 0, 0)
    d1, A1, B1, _, C1 = _gemm_operands(A1, B1, 1.0, 0.0, None, None, 0, 0)
    lib = L.lib()
    nb = lib.fiode_gemm_pair_workspace_bytes(ct.byref(d0), ct.byref(d1))
    ws = _gemm_ws(dev, nb) if nb else None
    L.check(lib.fiode_gemm_pair(_stream(dev), ct.byref(d0), A0.data_ptr(), B0.data_ptr(), None, C0.data_ptr(),
                                ct.byref(d1), A1.data_ptr(), B1.data_ptr(), None, C1.data_ptr(), _ptr(ws),
                                ws.numel() if ws is not None else 0), "fiode_gemm_pair")
    return C0, C1


def spectral_config(weight_shape, n: int) -> L.SpectralConfig:
    cout, cin, kh, kw = weight_shape
    if kh != kw:
        raise ValueError(f"spectral Cayley: square kernels only, got {kh}x{kw}")
    return L.SpectralConfig(int(cout), int(cin), int(kh), int(n))


def spectral_supported(weight_shape, n: int) -> bool:
    """Whether fiode_spectral_cayley_* takes this layer (3x3 taps, min(cout, cin) <= 64, the LDS
    image of one frequency within 160 KiB)."""
    cfg = spectral_config(weight_shape, n)
    return L.lib().fiode_spectral_workspace_bytes(ct.byref(cfg)) > 0


def spectral_cayley_forward(weight: torch.Tensor, alpha: torch.Tensor, n: int, out=None):
    """fiode_spectral_cayley_forward: Q complex64 [n (n/2+1), cout, cin] = cayley(alpha Wf / ||Wf||)
    per rFFT frequency.  Returns (Q, inv, workspace); inv and workspace feed the backward.  ``out``:
    a previous call's (Q, inv, workspace) to overwrite (a map computed ahead into fixed buffers)."""
    dev = weight.device
    cout, cin = int(weight.shape[0]), int(weight.shape[1])
    weight = _need(weight, "weight", tuple(weight.shape), torch.float32, dev)
    alpha = _need(alpha.reshape(1), "alpha", (1,), torch.float32, dev)
    cfg = spectral_config(weight.shape, n)
    lib = L.lib()
    nb = lib.fiode_spectral_workspace_bytes(ct.byref(cfg))
    if nb == 0:
        raise ValueError(f"spectral Cayley: unsupported layer {tuple(weight.shape)} at n={n}")
    nf, K = n * (n // 2 + 1), min(cout, cin)
    if out is not None:
        Q, inv, ws = out
        _need(Q, "Q", (nf, cout, cin), torch.complex64, dev)
        _need(inv, "inv", (nf, K, K), torch.complex64, dev)
        if ws.numel() < nb or not Q.is_contiguous() or not inv.is_contiguous():
            raise ValueError("spectral Cayley: out buffers too small or not contiguous")
    else:
        Q = torch.empty((nf, cout, cin), dtype=torch.complex64, device=dev)
        inv = torch.empty((nf, K, K), dtype=torch.complex64, device=dev)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    L.check(lib.fiode_spectral_cayley_forward(_stream(dev), ct.byref(cfg), weight.data_ptr(), alpha.data_ptr(),
                                              Q.data_ptr(), inv.data_ptr(), ws.data_ptr(), ws.numel()),
            "fiode_spectral_cayley_forward")
    return Q, inv, ws


def spectral_cayley_backward(gQ: torch.Tensor, weight: torch.Tensor, alpha: torch.Tensor, n: int,
                             inv: torch.Tensor, ws: torch.Tensor):
    """fiode_spectral_cayley_backward: (dL/dweight, dL/dalpha) from dL/dQ (torch's complex convention)."""
    dev = weight.device
    cout, cin = int(weight.shape[0]), int(weight.shape[1])
    nf = n * (n // 2 + 1)
    gQ = _need(gQ, "gQ", (nf, cout, cin), torch.complex64, dev)
    weight = _need(weight, "weight", tuple(weight.shape), torch.float32, dev)
    alpha = _need(alpha.reshape(1), "alpha", (1,), torch.float32, dev)
    cfg = spectral_config(weight.shape, n)
    gw = torch.empty_like(weight)
    ga = torch.empty(1, dtype=torch.float32, device=dev)
    L.check(L.lib().fiode_spectral_cayley_backward(_stream(dev), ct.byref(cfg), weight.data_ptr(), alpha.data_ptr(),
                                                   gQ.data_ptr(), inv.data_ptr(), gw.data_ptr(), ga.data_ptr(),
                                                   ws.data_ptr(), ws.numel()),
            "fiode_spectral_cayley_backward")
    return gw, ga


def _gs_shape(x: torch.Tensor, cdim: int = 1):
    if x.device.type != "cuda" or x.dtype != torch.float32:
        raise ValueError(f"groupsort: float32 ROCm tensor expected, got {x.dtype} on {x.device}")
    cdim = cdim % x.dim()
    outer = 1
    for d in x.shape[:cdim]:
        outer *= d
    Cc = x.shape[cdim]
    inner = 1
    for d in x.shape[cdim + 1:]:
        inner *= d
    if Cc % 2 or ((Cc // 2) * inner) % 4:
        raise ValueError(f"groupsort: shape {tuple(x.shape)} needs even C and (C/2)*inner % 4 == 0")
    return outer, Cc, inner


def groupsort_forward(x: torch.Tensor, cdim: int = 1) -> torch.Tensor:
    x = x.contiguous()
    B, Cc, S = _gs_shape(x, cdim)
    y = torch.empty_like(x)
    L.check(L.lib().fiode_groupsort_forward(_stream(x.device), B, Cc, S, x.data_ptr(), y.data_ptr()),
            "fiode_groupsort_forward")
    return y


def head_out(z: torch.Tensor, Q: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """fiode_head_out: z [B, K] Q [J, K]^T + bias [J] for J <= 16 (the head's output layer)."""
    dev = z.device
    B, K = z.shape
    J = Q.shape[0]
    z = _need(z, "z", (B, K), torch.float32, dev)
    Q = _need(Q.detach(), "Q", (J, K), torch.float32, dev)
    if bias is not None:
        bias = _need(bias.detach(), "bias", (J,), torch.float32, dev)
    out = torch.empty((B, J), dtype=torch.float32, device=dev)
    L.check(L.lib().fiode_head_out(_stream(dev), B, K, J, z.data_ptr(), Q.data_ptr(), _ptr(bias), out.data_ptr()),
            "fiode_head_out")
    return out


def head_out_backward_gs(g: torch.Tensor, Q: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """fiode_head_out_backward_gs: GroupSort backward (pre-activation y [B, K]) of g [B, J] Q [J, K]."""
    dev = g.device
    B, J = g.shape
    K = Q.shape[1]
    g = _need(g, "g", (B, J), torch.float32, dev)
    Q = _need(Q.detach(), "Q", (J, K), torch.float32, dev)
    y = _need(y, "y", (B, K), torch.float32, dev)
    gx = torch.empty((B, K), dtype=torch.float32, device=dev)
    L.check(L.lib().fiode_head_out_backward_gs(_stream(dev), B, K, J, g.data_ptr(), Q.data_ptr(), y.data_ptr(),
                                               gx.data_ptr()), "fiode_head_out_backward_gs")
    return gx


def groupsort_backward(x: torch.Tensor, g: torch.Tensor, cdim: int = 1) -> torch.Tensor:
    x, g = x.contiguous(), g.contiguous()
    B, Cc, S = _gs_shape(x, cdim)
    gx = torch.empty_like(x)
    L.check(L.lib().fiode_groupsort_backward(_stream(x.device), B, Cc, S, x.data_ptr(), g.data_ptr(), gx.data_ptr()),
            "fiode_groupsort_backward")
    return gx
