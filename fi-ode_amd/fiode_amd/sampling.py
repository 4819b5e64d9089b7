"""Samplers and sampler schedulers (sampling/sampler.py, sampling/sampler_schedulers.py).

The schedulers are host-side float64 scalar logic, restated exactly (they decide the per-step
S1/S2 split).  The samplers are descriptors: the fused Lyapunov step draws the samples itself
(in-kernel Philox, ``k_lyap_prep``), so ``CompositeSampler.kernel_plan`` turns the mixer into the
kernel's (sampler kind, n_uniform).  ``TrajectorySampler`` rows come from the HIP ODE solve and
reach the kernel as a [B, S - n_uniform, C] input (sampler kind TRAJECTORY).
"""
from __future__ import annotations

from math import floor
from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L


class AbstractScheduler:
    def sampler_weight(self, epoch_num):
        raise NotImplementedError(f"{type(self).__name__} defines no schedule value")


class LinearScheduler(AbstractScheduler):
    """sampler_schedulers.py:14-38."""

    def __init__(self, rate, bias=0.0, clamp="min", clamp_val=0.0, start=0):
        assert clamp_val >= 0, "a schedule value below zero"
        self.rate, self.bias, self.clamp, self.clamp_val, self.start = rate, bias, clamp, clamp_val, start

    def sampler_weight(self, epoch_num):
        if epoch_num < self.start:
            return 0.0 if self.rate > 0 else 1.0
        weight = (epoch_num - self.start) * self.rate + self.bias
        if self.clamp not in ("min", "max"):
            return weight
        return min(weight, self.clamp_val) if self.clamp == "max" else max(weight, self.clamp_val)


class ConstantScheduler(AbstractScheduler):
    """sampler_schedulers.py:41-48."""

    def __init__(self, constant):
        assert constant >= 0, "a schedule value below zero"
        self.constant = constant

    def sampler_weight(self, epoch_num):
        return self.constant


class SwitchScheduler(AbstractScheduler):
    """sampler_schedulers.py:50-63."""

    def __init__(self, start, end, trigger):
        assert start >= 0 and end >= 0, "a schedule value below zero"
        self.start, self.end, self.trigger = start, end, trigger

    def sampler_weight(self, epoch_num):
        return self.start if epoch_num < self.trigger else self.end


class CompositeSamplerScheduler:
    """sampler_schedulers.py:65-77: float64 L1 normalisation with +1e-12."""

    def __init__(self, schedulers, scheduler_weights):
        assert len(schedulers) == len(scheduler_weights), f"{len(schedulers)} schedules but {len(scheduler_weights)} weights"
        self.schedulers = list(schedulers)
        self.scheduler_weights = np.array(scheduler_weights, dtype=np.float64)

    def get_mixer_coefficients(self, epoch_num):
        c = np.array([s.sampler_weight(epoch_num) for s in self.schedulers], dtype=np.float64) * self.scheduler_weights
        return c / (np.linalg.norm(c, ord=1) + 1e-12)


class AbstractSampler(nn.Module):
    def __init__(self, h_dims=(10,)):
        super().__init__()
        self.h_dims = tuple(h_dims)

    def device_initialize(self, device):
        self.device = device


class UniformSimplexSampling(AbstractSampler):
    """Dirichlet(1) rows shared across the batch (sampler.py:24-38)."""


class CorrectConeSampling(AbstractSampler):
    """Dirichlet(1) rows with the label moved to the argmax (sampler.py:104-128)."""


class DecisionBoundarySampling(AbstractSampler):
    """Rows on the label's decision boundary (sampler.py:130-153)."""


class TrajectorySampler(AbstractSampler):
    """States along the ODE solve (sampler.py:156-166): ``model.model(x, ts=linspace(0, t_max, n),
    int_params=train_solver_params, return_traj=True)`` under no_grad, transposed to [B, n, C].

    The solve runs on libfiode: in eval mode (or dropout 0) the HIP stepper ``fiode_odeint``
    (rk4 / dopri5 dense output at the n times); in train mode with the fixed-grid rk4 solver, the
    train-mode solve ``fiode_odetrain_forward`` (fresh Philox dropout masks per f-eval, as the
    reference's dropout draws fresh masks per call), whose saved stage-1 inputs are the grid states,
    then torchdiffeq's FixedGridODESolver linear interpolation to the n output times.  A train-mode
    adaptive solve with dropout is not fused and raises."""

    TRAJ_SEED_SALT = 0x7A5C_3E11       # decorrelates its dropout masks from the train_ode solve's

    def trajectory(self, module, static_state: torch.Tensor, n: int) -> torch.Tensor:
        from . import ops
        from .odeint import _rk4_grid
        dyn = module.dyn_fun
        dev = static_state.device
        B = static_state.shape[0]
        h0 = module.init_coordinates.h0_0[None].expand(B, -1).float().contiguous()
        x = static_state.detach().float().contiguous()
        params = module.train_solver_params
        ts = torch.linspace(0.0, float(module.t_max), n)            # float32, as the reference builds it
        with torch.no_grad():
            w = {k: v.detach().float().contiguous() for k, v in dyn.effective_weights().items()}
            if not (dyn.training and dyn.dropout.p > 0):
                sol, _, _ = ops.odeint_dyn(x, h0, ts.to(dev, torch.float64), w, dyn.dyn_cfg(),
                                           method=params["method"], rtol=float(params.get("rtol", 1e-7)),
                                           atol=float(params.get("atol", 1e-9)),
                                           step_size=params.get("options", {}).get("step_size"))
                return sol.transpose(0, 1).contiguous()
            if params["method"] != "rk4":
                raise NotImplementedError("TrajectorySampler in train mode with dropout needs the fixed-grid rk4 "
                                          "train solver (the HIP train-mode solve); adaptive + dropout is not fused")
            step = float(params["options"]["step_size"])
            cfg = ops.odetrain_config(B, 0.0, float(module.t_max), step, L.FIODE_DROPOUT_PHILOX,
                                      seed=(module.seed ^ self.TRAJ_SEED_SALT),
                                      offset=module._rng_offset if module.rng_counter is None else 0)
            y1, _, ws = ops.odetrain_forward(x, h0, w, dyn.dyn_cfg(), cfg, offset_dev=module.rng_counter)
            saved = ops.odetrain_saved(ws, cfg)
            grid_states = torch.cat([saved["h"][:, 0::4], y1[:, None]], dim=1)       # [B, niters, C]
            grid = _rk4_grid(ts[0], ts[-1], step, torch.float32)
            assert grid.numel() == grid_states.shape[1]
            k, slope, pick = fixed_grid_interp_plan(grid, ts)
            k_t = torch.from_numpy(k).to(dev)
            ya, yb = grid_states[:, k_t], grid_states[:, k_t + 1]
            out = ya + torch.from_numpy(slope).to(dev)[None, :, None] * (yb - ya)
            pick_t = torch.from_numpy(pick).to(dev)[None, :, None]
            out = torch.where(pick_t == 1, ya, torch.where(pick_t == 2, yb, out))
            return out.contiguous()


def fixed_grid_interp_plan(grid: torch.Tensor, t: torch.Tensor):
    """FixedGridODESolver's output rule (torchdiffeq 0.2.2, as restated in odeint._odeint_torch):
    t[0] is y0; every later t[j] is served by the first grid interval (ta, tb] with tb >= t[j]:
    t[j] == ta -> y(ta), t[j] == tb -> y(tb), else y(ta) + (t[j]-ta)/(tb-ta) (y(tb) - y(ta)) in float32.
    Returns (interval index k[n], slope float32[n], pick int8[n]: 0 lerp, 1 y(ta), 2 y(tb))."""
    g = grid.to(torch.float32).numpy()
    tt = t.to(torch.float32).numpy()
    n = tt.shape[0]
    k = np.zeros(n, dtype=np.int64)
    slope = np.zeros(n, dtype=np.float32)
    pick = np.ones(n, dtype=np.int8)                 # t[0]: y0 = grid state 0
    j = 1
    for i in range(g.shape[0] - 1):
        ta, tb = g[i], g[i + 1]
        while j < n and tb >= tt[j]:
            k[j] = i
            if tt[j] == ta:
                pick[j] = 1
            elif tt[j] == tb:
                pick[j] = 2
            else:
                pick[j] = 0
                slope[j] = np.float32((tt[j] - ta) / (tb - ta))
            j += 1
    if j < n:
        raise ValueError("output times beyond the solve's grid")
    return k, slope, pick


class CompositeSampler(nn.Module):
    """sampler.py:169-216."""

    def __init__(self, h_dims, samplers):
        super().__init__()
        self.samplers = list(samplers)
        self.h_dims = tuple(h_dims)

    def device_initialize(self, device):
        for s in self.samplers:
            s.device_initialize(device)

    @staticmethod
    def _coefficient_to_num_samples(sample_size, mixer_coefficients) -> List[int]:
        """sampler.py:181-192."""
        mixed, added = [], 0
        for coeff in mixer_coefficients:
            if len(mixed) == len(mixer_coefficients) - 1:
                mixed.append(sample_size - added)
                break
            s = floor(sample_size * coeff)
            added += s
            mixed.append(s)
        assert sum(mixed) == sample_size
        return mixed

    def kernel_plan(self, sample_size: int, mixer_coefficients: Sequence[float]) -> Tuple[int, int]:
        """(fiode sampler kind, n_uniform) for the fused step."""
        assert len(mixer_coefficients) == len(self.samplers), f"{len(self.samplers)} samplers but {len(mixer_coefficients)} mixer coefficients"
        assert abs(sum(mixer_coefficients) - 1.0) < 1e-8, f"mixer coefficients sum to {sum(mixer_coefficients)}, not 1"
        split = self._coefficient_to_num_samples(sample_size, mixer_coefficients)
        kinds = [type(s) for s in self.samplers]
        if kinds == [UniformSimplexSampling, CorrectConeSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, split[0]
        if kinds == [CorrectConeSampling, UniformSimplexSampling]:
            raise NotImplementedError("the fused sampler orders Uniform rows before CorrectCone rows")
        if all(k is DecisionBoundarySampling for k in kinds):
            return L.FIODE_SAMPLER_DECISION_BOUNDARY, 0
        if kinds == [UniformSimplexSampling, TrajectorySampler]:
            return L.FIODE_SAMPLER_TRAJECTORY, split[0]
        if kinds == [TrajectorySampler]:
            return L.FIODE_SAMPLER_TRAJECTORY, 0
        if kinds == [UniformSimplexSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, sample_size
        if kinds == [CorrectConeSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, 0
        raise NotImplementedError(f"sampler mix {kinds} is not fused (SURVEY.md section 2 row 6b)")
