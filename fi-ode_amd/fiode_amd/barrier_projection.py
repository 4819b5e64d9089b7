"""FastBarrierProjectionNoUpper over the C ABI (barrier_projection.py:217-313).

Same factory signature as the reference: ``FastBarrierProjectionNoUpper(max_iter, tol, verbose)``
returns an ``apply(lower, nominal) -> v`` whose forward is the bisection with the batch-global exit
(no host syncs: the exit iteration is found on the device) and whose backward is the reference's
dense-mask Jacobian in closed form (O(C) per row).
"""
from __future__ import annotations

import torch

from . import ops


def FastBarrierProjectionNoUpper(max_iter=10, tol=1e-4, verbose=False):
    class BarrierProjectionFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, lower, nominal):
            v, mu, it = ops.qp_forward(lower.detach().float().contiguous(), nominal.detach().float().contiguous(),
                                       max_iter=max_iter, tol=tol)
            ctx.save_for_backward(v, mu, lower.detach(), nominal.detach())
            ctx.exit_iter = it
            return v

        @staticmethod
        def backward(ctx, g):
            v, mu, lower, nominal = ctx.saved_tensors
            g_lower, g_nominal = ops.qp_backward(g.float().contiguous(), v, mu, lower.float().contiguous(),
                                                 nominal.float().contiguous())
            return g_lower, g_nominal

    return BarrierProjectionFn.apply
