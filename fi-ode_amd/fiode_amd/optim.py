"""Adam / AdamW whose update is one HIP launch over every parameter tensor (adam.hip).

The reference's optimizer is torch.optim.Adam / AdamW (pl_modules.py:97-147 configure_optimizers).
FiodeAdam / FiodeAdamW ARE those classes (subclasses: same constructor, param groups, state layout
and ``state_dict`` -- checkpoints load either way); only ``step()`` differs: the step counts are
incremented as torch does, then ``fiode_adam_step`` applies torch's fused Adam formula to all
float32 ROCm tensors of a param group in a single launch (torch's fused multi-tensor Adam is ~3
launches and ~50 us for the KWLarge model's 2.6 M parameters; this one streams p/g/m/v once).

A tensor lr (torch's way to schedule the learning rate under graph capture: LR schedulers update
it in place) is read by the kernel on the device, so a captured step follows the schedule; a float
lr is a launch argument, baked into a captured graph (GraphTrainStep refuses to replay after it
changed).  Groups the kernel does not cover (CPU or non-float32 parameters, amsgrad,
differentiable, more than FIODE_ADAM_MAX_TENSORS tensors, a tensor lr off the parameters' device)
go through torch's own Adam.step unchanged.

Step guard (``opt.guard = StepGuard(...)``): the kernel reads, on the device, whether this step
may touch the parameters -- the train_ode solve's status words, the loss's finiteness, or (N
ranks) the guard slot of the all-reduced gradient bucket -- and otherwise leaves p, m, v and the
device step counts as they were, counting the skipped step in a sticky device word (torch.amp's
found_inf skip, decided without a host sync; GraphTrainStep arms it).
"""
from __future__ import annotations

import ctypes as ct
from typing import List

import torch

from . import _lib as L
from .ops import _stream

MAX_TENSORS = 64          # FIODE_ADAM_MAX_TENSORS (include/fiode.h)


def _kernel_ok(group, params: List[torch.Tensor]) -> bool:
    if group["amsgrad"] or group["differentiable"]:
        return False
    if not params or len(params) > MAX_TENSORS:
        return False
    dev = params[0].device
    lr = group["lr"]
    if torch.is_tensor(lr) and (lr.device != dev or lr.numel() != 1 or lr.dtype not in (torch.float32, torch.float64)):
        return False
    for p in params:
        g = p.grad
        if (p.device != dev or dev.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous()
                or g is None or g.is_sparse or g.dtype != torch.float32 or not g.is_contiguous()
                or g.device != dev):
            return False
    return True


def _kernel_ok_params(opt, params: List[torch.Tensor]) -> bool:
    """Whether the kernel will cover these parameters' updates (group settings, placement, dtype;
    gradients are not looked at): what step_params needs."""
    if not isinstance(opt, _KernelStepMixin):
        return False
    ids = {id(p) for p in params}
    for group in opt.param_groups:
        sel = [p for p in group["params"] if id(p) in ids]
        if not sel:
            continue
        if group["amsgrad"] or group["differentiable"] or len(group["params"]) > MAX_TENSORS:
            return False
        dev = sel[0].device
        lr = group["lr"]
        if torch.is_tensor(lr) and (lr.device != dev or lr.numel() != 1
                                    or lr.dtype not in (torch.float32, torch.float64)):
            return False
        if any(p.device != dev or dev.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous()
               for p in sel):
            return False
        ids -= {id(p) for p in sel}
    return not ids


class StepGuard:
    """Device-side skip condition of an optimizer step (include/fiode.h fiode_step_guard): skip when
    ``flag`` (float32 [1]) is nonzero or NaN, ``loss`` is not finite, or any ``status`` word (int32
    [1]) is nonzero; ``skipped`` (int32 [1]) counts the skipped steps.  Keeps the tensors alive."""

    def __init__(self, flag=None, loss=None, status=(), skipped=None):
        status = [t for t in status if t is not None]
        if len(status) > L.FIODE_GUARD_MAX_STATUS:
            raise ValueError(f"at most {L.FIODE_GUARD_MAX_STATUS} status words")
        for t, dt in [(flag, torch.float32), (loss, torch.float32), (skipped, torch.int32)] + \
                [(t, torch.int32) for t in status]:
            if t is not None and (t.dtype != dt or not t.is_cuda or t.numel() < 1):
                raise ValueError(f"StepGuard: expected a {dt} device tensor, got {t.dtype} on {t.device}")
        self.flag, self.loss, self.status, self.skipped = flag, loss, status, skipped

    def to_c(self, count: bool = True) -> "L.StepGuard":
        ptr = lambda t: None if t is None else t.data_ptr()
        st = (ct.c_void_p * L.FIODE_GUARD_MAX_STATUS)(*([t.data_ptr() for t in self.status] +
                                                         [None] * (L.FIODE_GUARD_MAX_STATUS - len(self.status))))
        return L.StepGuard(ptr(self.flag), ptr(self.loss), st, ptr(self.skipped) if count else None)

    def write_flag(self, out: torch.Tensor) -> None:
        """out[0] = 1.0 if this rank's loss / status words say skip, else 0.0 (fiode_step_guard_flag),
        on the current stream -- the value that goes into the all-reduced guard slot."""
        g = self.to_c(count=False)
        L.check(L.lib().fiode_step_guard_flag(_stream(out.device), ct.byref(g), out.data_ptr()),
                "fiode_step_guard_flag")


class _KernelStepMixin:
    _decoupled = False
    guard = None          # StepGuard or None

    def _done_set(self) -> set:
        d = self.__dict__.get("_fiode_done")
        if d is None:
            d = self.__dict__["_fiode_done"] = set()
        return d

    @torch.no_grad()
    def step_params(self, pairs) -> None:
        """Update only the given (parameter, gradient) pairs now, with their groups' settings and
        the same kernel as step(); the next step() skips them (it updates the rest and clears the
        marks).  For updating a layer as soon as its gradient is final (GraphTrainStep's maps
        computed ahead).  The parameters must be covered by the kernel (ROCm float32, ...)."""
        done = self._done_set()
        for group in self.param_groups:
            ids = {id(p) for p in group["params"]}
            sel = [(p, g) for p, g in pairs if id(p) in ids]
            if not sel:
                continue
            saved = [p.grad for p, _ in sel]
            try:
                for p, g in sel:
                    p.grad = g
                params = [p for p, _ in sel]
                if not _kernel_ok(group, params):
                    raise RuntimeError("FiodeAdam.step_params: parameters not covered by the kernel")
                pw, grads, m, v, mx, steps = [], [], [], [], [], []
                self._init_group({**group, "params": params}, pw, grads, m, v, mx, steps)
                if not self._launch(group, pw, grads, m, v, steps, count_skip=False):
                    raise RuntimeError("FiodeAdam.step_params: the parameters' step counts differ")
            finally:
                for (p, _), g0 in zip(sel, saved):
                    p.grad = g0
            done.update(id(p) for p, _ in sel)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        fallback = []
        counted = False
        done = self._done_set()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None and id(p) not in done]
            if not params:
                continue
            if not _kernel_ok(group, params):
                if done:
                    raise RuntimeError("FiodeAdam: torch fallback after step_params is not supported")
                fallback.append(group)
                continue
            pw, grads, m, v, mx, steps = [], [], [], [], [], []
            self._init_group({**group, "params": params}, pw, grads, m, v, mx, steps)   # torch's lazy state creation
            if self._launch(group, pw, grads, m, v, steps, count_skip=not counted):
                counted = True              # a skipped step is counted once, not once per group
            else:
                if done:
                    raise RuntimeError("FiodeAdam: host step counts after step_params are not supported")
                fallback.append(group)
        done.clear()
        if fallback:
            kept = self.param_groups
            self.param_groups = fallback
            try:
                super().step()
            finally:
                self.param_groups = kept
        return loss

    def _launch(self, group, pw, grads, m, v, steps, count_skip: bool = True) -> bool:
        """The kernel update of one group's tensors; False (nothing done) when the host step counts
        cannot take it (mixed placement or counts: torch's path).  Device step counts are
        incremented by the library (guarded: a skipped step leaves them)."""
        n = len(pw)
        on_dev = [s.device.type == "cuda" for s in steps]
        if all(on_dev):
            if any(s.dtype != torch.float32 for s in steps):
                return False
            host_step = 0.0
        else:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FiodeAdam: capturing the step in a graph needs capturable=True "
                                   "(device step counts)")
            if any(on_dev) or len({float(s) for s in steps}) != 1:
                return False                    # mixed step placement / counts: torch's path
            if self.guard is not None:
                # the host would count the step before the device decides to skip it, so a skipped
                # step would still move the bias correction: guarded steps need device counts
                raise RuntimeError("FiodeAdam: a step guard needs device step counts (capturable=True)")
            for s in steps:
                s += 1
            host_step = float(steps[0])
        beta1, beta2 = group["betas"]
        lr = group["lr"]
        lr_t = lr if torch.is_tensor(lr) else None
        cfg = L.AdamConfig(n, int(bool(group.get("decoupled_weight_decay", self._decoupled))),
                           int(group["maximize"]), int(all(on_dev)), 0.0 if lr_t is not None else float(lr),
                           float(beta1),
                           float(beta2), float(group["eps"]), float(group["weight_decay"]), host_step,
                           lr_t.data_ptr() if lr_t is not None else None,
                           int(lr_t is not None and lr_t.dtype == torch.float64), 0)
        arr = ct.c_void_p * n
        step_ptrs = arr(*[s.data_ptr() for s in steps]) if all(on_dev) else None
        guard = self.guard.to_c(count=count_skip) if self.guard is not None else None
        L.check(L.lib().fiode_adam_step(
            _stream(pw[0].device), ct.byref(cfg), arr(*[t.data_ptr() for t in pw]),
            arr(*[t.data_ptr() for t in grads]), arr(*[t.data_ptr() for t in m]),
            arr(*[t.data_ptr() for t in v]), (ct.c_int64 * n)(*[t.numel() for t in pw]), step_ptrs,
            ct.byref(guard) if guard is not None else None), "fiode_adam_step")
        return True


class FiodeAdam(_KernelStepMixin, torch.optim.Adam):
    """torch.optim.Adam with the one-launch HIP update (same arguments and state)."""


class FiodeAdamW(_KernelStepMixin, torch.optim.AdamW):
    """torch.optim.AdamW with the one-launch HIP update (same arguments and state)."""
    _decoupled = True
