"""Samplers and sampler schedulers (sampling/sampler.py, sampling/sampler_schedulers.py).

The schedulers are host-side float64 scalar logic, restated exactly (they decide the per-step
S1/S2 split).  The samplers are descriptors: the fused Lyapunov step draws the samples itself
(in-kernel Philox, ``k_lyap_prep``), so ``CompositeSampler.kernel_plan`` turns the mixer into the
kernel's (sampler kind, n_uniform).  ``CompositeSampler.forward`` keeps the reference signature
for callers that want the samples as a tensor (it runs the same kernel with debug output).
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
        raise NotImplementedError("[ERROR] Not Implemented")


class LinearScheduler(AbstractScheduler):
    """sampler_schedulers.py:14-38."""

    def __init__(self, rate, bias=0.0, clamp="min", clamp_val=0.0, start=0):
        assert clamp_val >= 0, "Schedulers must return positive number"
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
        assert constant >= 0, "Schedulers must return positive number"
        self.constant = constant

    def sampler_weight(self, epoch_num):
        return self.constant


class SwitchScheduler(AbstractScheduler):
    """sampler_schedulers.py:50-63."""

    def __init__(self, start, end, trigger):
        assert start >= 0 and end >= 0, "Schedulers must return positive number"
        self.start, self.end, self.trigger = start, end, trigger

    def sampler_weight(self, epoch_num):
        return self.start if epoch_num < self.trigger else self.end


class CompositeSamplerScheduler:
    """sampler_schedulers.py:65-77: float64 L1 normalisation with +1e-12."""

    def __init__(self, schedulers, scheduler_weights):
        assert len(schedulers) == len(scheduler_weights), "each scheduler needs a weight"
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
        assert len(mixer_coefficients) == len(self.samplers), "[ERROR] Each sampler must have a mixer coefficient"
        assert abs(sum(mixer_coefficients) - 1.0) < 1e-8, "[ERROR] mixer coefficeints need to sum to one."
        split = self._coefficient_to_num_samples(sample_size, mixer_coefficients)
        kinds = [type(s) for s in self.samplers]
        if kinds == [UniformSimplexSampling, CorrectConeSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, split[0]
        if kinds == [CorrectConeSampling, UniformSimplexSampling]:
            raise NotImplementedError("the fused sampler orders Uniform rows before CorrectCone rows")
        if all(k is DecisionBoundarySampling for k in kinds):
            return L.FIODE_SAMPLER_DECISION_BOUNDARY, 0
        if kinds == [UniformSimplexSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, sample_size
        if kinds == [CorrectConeSampling]:
            return L.FIODE_SAMPLER_COMPOSITE, 0
        raise NotImplementedError(f"sampler mix {kinds} is not fused (SURVEY.md section 2 row 6b)")
