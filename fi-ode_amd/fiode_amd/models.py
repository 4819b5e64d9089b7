"""Backbone (param_map) and IVP wrapper.

``Normalize`` + ``make_ortho_KWLarge_Concat`` mirror models.py:17-35 of the reference.  The
KWLarge_Concat body lives in the absent ``libs/ortho_conv`` submodule; it is restated here from
the public KWLarge design (4 Cayley convs with GroupSort, 3 Cayley linears) with ``out_dim``
outputs -- parity unpinned, and it stays PyTorch-ROCm host code (the
backbone as HIP/MFMA is the next row after the fan-out path).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn

from .cayley import CayleyConv, CayleyLinear, GroupSort


class Normalize(nn.Module):
    """(x - mu) / std per channel (models.py:17-26)."""

    def __init__(self, mu: Sequence[float], std: Optional[Sequence[float]]):
        super().__init__()
        self.register_buffer("mu", torch.tensor(list(mu), dtype=torch.float32).view(-1, 1, 1))
        self.register_buffer("std", None if std is None else torch.tensor(list(std), dtype=torch.float32).view(-1, 1, 1))

    def forward(self, x):
        if self.std is not None:
            return (x - self.mu) / self.std
        return x - self.mu


class KWLargeConcat(nn.Module):
    """KWLarge-shaped Cayley-orthogonal CIFAR backbone -> out_dim features."""

    def __init__(self, out_dim: int = 10, act: str = "GroupSort", w: int = 1):
        super().__init__()
        act_fn = GroupSort if act == "GroupSort" else nn.ReLU
        self.model = nn.Sequential(
            CayleyConv(3, 32 * w, 3), act_fn(),
            CayleyConv(32 * w, 32 * w, 3, stride=2), act_fn(),
            CayleyConv(32 * w, 64 * w, 3), act_fn(),
            CayleyConv(64 * w, 64 * w, 3, stride=2), act_fn(),
            nn.Flatten(),
            CayleyLinear(4096 * w, 512 * w), act_fn(),
            CayleyLinear(512 * w, 512), act_fn(),
            CayleyLinear(512, out_dim),
        )

    def forward(self, x):
        return self.model(x)


def make_ortho_KWLarge_Concat(n_in_channels=3, n_outputs=10, mu=(0.485, 0.456, 0.406), std=(0.225, 0.225, 0.225),
                              out_dim=10, act="GroupSort"):
    """models.py:29-35 (CIFAR10 MU/STD from ExpConfig.py:57-58)."""
    return nn.Sequential(Normalize(mu, std), KWLargeConcat(out_dim=out_dim, act=act))
