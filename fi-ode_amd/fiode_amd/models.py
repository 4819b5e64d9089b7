"""Backbone (param_map) and IVP wrapper.

``Normalize`` + ``make_ortho_KWLarge_Concat`` mirror models.py:17-35 of the reference.  The
KWLarge_Concat body lives in the absent ``libs/ortho_conv`` submodule; it is restated here from
the public KWLarge design (4 Cayley convs with GroupSort, 3 Cayley linears) with ``out_dim``
outputs -- parity unpinned.  On ROCm tensors its per-layer work runs in libfiode.so (SURVEY.md
section 8f row f1: spectral Cayley maps, the conv transforms + GroupSort, the dense Cayley stages
and block inverses; cayley.py); the complex / dense GEMMs stay on hipBLASLt, and host tensors
take the PyTorch formula.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn

from .cayley import CayleyConv, CayleyLinear, GroupSort, linear_head


class Normalize(nn.Module):
    """(x - mu) / std per channel (models.py:17-26)."""

    def __init__(self, mu: Sequence[float], std: Optional[Sequence[float]]):
        super().__init__()
        self.register_buffer("mu", torch.tensor(list(mu), dtype=torch.float32).view(-1, 1, 1))
        self.register_buffer("std", None if std is None else torch.tensor(list(std), dtype=torch.float32).view(-1, 1, 1))

    fused_hwcb = True      # ROCm: one kernel that also lays the result out spatial-major (see forward)

    def forward(self, x):
        """On ROCm inputs that need no gradient, one kernel (fiode_normalize_hwcb) computes the same
        float32 (x - mu) / std and stores it spatial-major ([h, w, C, B], the conv stack's layout);
        the NCHW-shaped result is a view of that storage, so KWLargeConcat's permute to
        spatial-major is free.  Otherwise the two torch ops."""
        if self.fused_hwcb and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and not x.requires_grad:
            from . import _lib as L, ops
            B, C, H, W = x.shape
            xc = x.contiguous()
            y = torch.empty((H, W, C, B), dtype=torch.float32, device=x.device)
            mu = self.mu.reshape(-1).contiguous()
            sd = None if self.std is None else self.std.reshape(-1).contiguous()
            L.check(L.lib().fiode_normalize_hwcb(ops._stream(x.device), B, C, H, W, xc.data_ptr(), mu.data_ptr(),
                                                 None if sd is None else sd.data_ptr(), y.data_ptr()),
                    "fiode_normalize_hwcb")
            return y.permute(3, 2, 0, 1)
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

        self.spatial_major = True
        self.fused_transforms = True      # sconv.hip rfft2 / irfft2 (+ GroupSort) around the GEMMs
        self.nchw_last = True             # the last conv's transform writes the flatten's NCHW order

    def can_take_nchw(self, x) -> bool:
        """Whether forward(x, norm=...) can run the first conv straight from the NCHW input."""
        m = self.model[0]
        return (self.spatial_major and self.fused_transforms and x.is_cuda and x.dtype == torch.float32
                and x.dim() == 4 and not x.requires_grad and isinstance(m, CayleyConv) and not m.downsample
                and x.shape[-1] == x.shape[-2] and x.shape[-1] in (8, 16, 32))

    def forward(self, x, norm=None):
        """On ROCm the conv stack runs spatial-major ([h, w, C, B]: FFT and GEMM operands without
        permute copies, CayleyConv.forward_hwcb); the flatten restores the reference's (C, h, w)
        feature order.  Host tensors take the module-by-module NCHW path.  norm = (mu, sd): x is the
        raw NCHW input and the first conv applies the Normalize in its transform (NormalizedBackbone)."""
        if not (self.spatial_major and x.is_cuda):
            return self.model(x)
        mods = list(self.model)
        i = 0
        nconv = 0
        # after_conv_hook(conv index) -> None (e.g. a prefetch launch), re-read at every call site so a
        # hook may install the next one; index -1: input laid out, before the first conv
        if norm is not None:
            if getattr(self, "after_conv_hook", None) is not None:
                self.after_conv_hook(-1)
            gs = isinstance(mods[1], GroupSort)
            h = mods[0].forward_nchw_fused(x, norm[0], norm[1], gs)
            i = 2 if gs else 1
            if getattr(self, "after_conv_hook", None) is not None:
                self.after_conv_hook(0)
            nconv = 1
        else:
            h = x.permute(2, 3, 1, 0).contiguous()
            if getattr(self, "after_conv_hook", None) is not None:
                self.after_conv_hook(-1)
        nchw = False
        while not isinstance(mods[i], nn.Flatten):
            m = mods[i]
            if isinstance(m, CayleyConv):
                gs = i + 1 < len(mods) and isinstance(mods[i + 1], GroupSort)
                if self.fused_transforms and h.shape[0] // (2 if m.downsample else 1) <= 32:
                    # the last conv (+ GroupSort) writes NCHW: the flatten below is then a view
                    nchw = bool(self.nchw_last and gs and i + 2 < len(mods) and isinstance(mods[i + 2], nn.Flatten))
                    h = m.forward_hwcb_fused(h, gs, nchw_out=nchw)     # transforms (+ GroupSort) in HIP kernels
                    i += 2 if gs else 1
                    if getattr(self, "after_conv_hook", None) is not None:
                        self.after_conv_hook(nconv)
                    nconv += 1
                    continue
                h = m.forward_hwcb(h)
                if getattr(self, "after_conv_hook", None) is not None:
                    self.after_conv_hook(nconv)
                nconv += 1
            elif isinstance(m, GroupSort):
                h = m(h, channel_dim=2)
            else:
                h = m(h)
            i += 1
        h = h.reshape(h.shape[0], -1) if nchw else h.permute(3, 2, 0, 1).reshape(h.shape[3], -1)
        return linear_head(mods[i + 1:], h)


class NormalizedBackbone(nn.Sequential):
    """nn.Sequential(Normalize, KWLargeConcat) (the same modules and state-dict keys) whose forward on
    ROCm hands the raw NCHW input and the normalisation to the backbone's first conv transform
    (fiode_sconv_rfft2_nchw): the spatial-major normalised copy and its launch drop out.  Anything
    else runs the two modules in turn."""

    fused_input = True

    def forward(self, x):
        norm, net = self[0], self[1]
        if (self.fused_input and len(self) == 2 and isinstance(norm, Normalize) and isinstance(net, KWLargeConcat)
                and norm.fused_hwcb and net.can_take_nchw(x)):
            return net(x.contiguous(), norm=(norm.mu, norm.std))
        return super().forward(x)


def make_ortho_KWLarge_Concat(n_in_channels=3, n_outputs=10, mu=(0.485, 0.456, 0.406), std=(0.225, 0.225, 0.225),
                              out_dim=10, act="GroupSort"):
    """models.py:29-35 (CIFAR10 MU/STD from ExpConfig.py:57-58)."""
    return NormalizedBackbone(Normalize(mu, std), KWLargeConcat(out_dim=out_dim, act=act))


class DefaultOutputFun(nn.Module):
    """dynamics/output_coordinates.py:4-9."""

    def forward(self, h):
        return h[-1]


class IVP(nn.Module):
    """models.py:181-242: holds dyn_fun / init_coordinates / output_fun; ``integrate`` calls the
    torchdiffeq-compatible odeint, which runs the HIP solver for the HIP dynamics."""

    def __init__(self, n_input, n_output, dyn_fun, init_coordinates, output_fun=None, ode_tol=1e-2, ts=None):
        super().__init__()
        self.n_input = n_input
        self.n_output = n_output
        self.dyn_fun = dyn_fun
        self.ode_tol = ode_tol
        self.register_buffer("ts", torch.linspace(0, 1, 200) if ts is None else ts)
        self.output_fun = output_fun if output_fun is not None else DefaultOutputFun()
        self.init_coordinates = init_coordinates

    def h_dot(self, t, h):
        return self.dyn_fun.ode_forward(t, h)

    def forward(self, x, ts=None, int_params=None, use_adjoint=False, return_traj=False):
        solution = self.integrate(x, ts=ts, int_params=int_params, use_adjoint=use_adjoint)
        if return_traj:
            return self.output_fun(solution)
        return self.output_fun(solution)[-1]

    def integrate(self, x, ts=None, int_params=None, use_adjoint=False):
        from .odeint import odeint
        if use_adjoint:
            raise NotImplementedError("odeint_adjoint (SURVEY.md section 8f row 3)")
        ts = self.ts if ts is None else ts
        int_params = dict(rtol=self.ode_tol, atol=self.ode_tol) if int_params is None else dict(int_params)
        static_state, state = self.init_coordinates(x, self.dyn_fun)
        return self.integrate_from(static_state, state, ts=ts, int_params=int_params)

    def integrate_from(self, static_state, state, ts=None, int_params=None):
        """`integrate` from init_coordinates' outputs already in hand (the backbone is deterministic:
        a caller that needs both the features and the solve runs the backbone once)."""
        from .odeint import odeint
        ts = self.ts if ts is None else ts
        int_params = dict(rtol=self.ode_tol, atol=self.ode_tol) if int_params is None else dict(int_params)
        self.dyn_fun.static_state = static_state
        return odeint(self.h_dot, state, ts, **int_params)
