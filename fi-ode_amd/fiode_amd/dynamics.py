"""OrthoClassDynProjectSimplexLips with its per-sample work on the GPU (libfiode.so).

Mirror of dynamics/classification.py:31-132: same constructor fields, same submodule names and
state_dict keys (hidden_to_mlp / mlp_to_mlp / mlp_to_hidden / U_x with weight, bias, alpha;
buffer static_state), same methods.  ``eval_dot`` / ``eval_dot_light`` / ``ode_forward`` run the
fused HIP kernels (MLP + barrier + bisection QP with the reference's batch-global exit); the
training-mode eval_dot with dropout and autograd is fused into the Lyapunov step
(``fiode_amd.lyapunov``), which is the only place the reference differentiates it.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .cayley import CayleyLinear, cayley_scaled


class LipsLinear(nn.Linear):
    """nn.Linear with a ``singular_u`` buffer (classification.py:25-28)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.register_buffer("singular_u", None)

    def effective_weight(self):
        return self.weight


class OrthoClassDynProjectSimplexLips(nn.Module):
    def __init__(self, n_hidden=10, activation="ReLU", dropout=0.5, mlp_size=128, kappa=5.0, kappa_length=3e4,
                 alpha_1=100.0, alpha_2=5.0, sigma_1=0.02, scale_nominal=False, x_dim=10, cayley=True):
        super().__init__()
        if (n_hidden, mlp_size, x_dim) != (ops.C, ops.M, ops.X):
            raise NotImplementedError(f"libfiode is built for n_hidden=10, mlp_size=128, x_dim=10 "
                                      f"(got {n_hidden}, {mlp_size}, {x_dim})")
        if activation != "ReLU":
            raise NotImplementedError("the fused dynamics kernels implement activation='ReLU' "
                                      "(the README training/certify commands); GroupSort is not built")
        self.activation = nn.ReLU()
        self.dropout = nn.Dropout(dropout)
        self.mlp_size = mlp_size
        self.n_hidden = n_hidden
        self.kappa = kappa
        self.kappa_length = kappa_length
        self.register_buffer("static_state", None)
        self.alpha_1 = alpha_1
        self.alpha_2 = alpha_2
        self.sigma_1 = sigma_1
        self.qp_max_iter = 30          # FastBarrierProjectionNoUpper(max_iter=30, tol=1e-4), classification.py:63
        self.qp_tol = 1e-4
        self.scale_nominal = scale_nominal
        self.cayley = cayley
        lin = CayleyLinear if cayley else LipsLinear
        self.hidden_to_mlp = lin(n_hidden, mlp_size, bias=True)
        self.mlp_to_mlp = lin(mlp_size, mlp_size)
        self.mlp_to_hidden = lin(mlp_size, n_hidden)
        self.U_x = lin(x_dim, mlp_size)

    # -- parameters as the kernels take them ---------------------------------------------------
    def prefetch(self, stream) -> None:
        """Compute the next effective_weights() on a side stream (joined at the next call)."""
        from .cayley import _prefetch
        self._pre = _prefetch(stream, self._effective_weights)

    def effective_weights(self) -> Dict[str, torch.Tensor]:
        pre = getattr(self, "_pre", None)
        if pre is not None:
            from .cayley import _take
            self._pre = None
            return _take(pre)
        return self._effective_weights()

    def _effective_weights(self) -> Dict[str, torch.Tensor]:
        """Q = cayley(alpha W / ||W||) for each layer (differentiable), with the biases.  The three
        128x10-shaped maps (hidden_to_mlp, U_x and the transpose of mlp_to_hidden) run as one
        batched Cayley map (per-matrix norms and alphas); mlp_to_mlp on its own."""
        if self.cayley:
            l1, lx, l3 = self.hidden_to_mlp, self.U_x, self.mlp_to_hidden
            Wb = torch.stack([l1.weight, lx.weight, l3.weight.t()])
            ab = torch.cat([l1.alpha, lx.alpha, l3.alpha])
            Qb = cayley_scaled(Wb, ab, per_matrix=True)
            # Q3 made contiguous here (on the maps' prefetch stream): the solve and the fan-out read
            # it contiguous, and the copy otherwise ran on the step's chain right before the solve
            Q3 = Qb[2].t().contiguous()
            return {"Q1": Qb[0], "b1": l1.bias, "Qx": Qb[1], "bx": lx.bias,
                    "Q2": self.mlp_to_mlp.effective_weight(), "b2": self.mlp_to_mlp.bias,
                    "Q3": Q3, "b3": l3.bias}
        return {"Q1": self.hidden_to_mlp.effective_weight(), "b1": self.hidden_to_mlp.bias,
                "Qx": self.U_x.effective_weight(), "bx": self.U_x.bias,
                "Q2": self.mlp_to_mlp.effective_weight(), "b2": self.mlp_to_mlp.bias,
                "Q3": self.mlp_to_hidden.effective_weight(), "b3": self.mlp_to_hidden.bias}

    def dyn_cfg(self) -> ops.DynCfg:
        return ops.DynCfg(alpha_1=self.alpha_1, alpha_2=self.alpha_2, sigma_1=self.sigma_1,
                          scale_nominal=bool(self.scale_nominal), dropout=float(self.dropout.p),
                          qp_max_iter=self.qp_max_iter, qp_tol=self.qp_tol)

    # -- reference methods ----------------------------------------------------------------------
    def _h_dot_raw(self, h, x):
        """classification.py:96-102 (used by the optional barrier loss; PyTorch ops on device)."""
        w = self.effective_weights()
        z = F.linear(h, w["Q1"], w["b1"]) + F.linear(x, w["Qx"], w["bx"])
        z = self.activation(self.dropout(z))
        z = self.activation(self.dropout(F.linear(z, w["Q2"], w["b2"])))
        return F.linear(z, w["Q3"], w["b3"])

    def _eval(self, h: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        if self.training and self.dropout.p > 0:
            raise NotImplementedError("training-mode eval_dot (dropout) is fused into LyapunovLearning.compute_loss")
        if torch.is_grad_enabled() and (h.requires_grad or x.requires_grad):
            raise NotImplementedError("eval_dot is differentiated only inside the fused Lyapunov step")
        with torch.no_grad():
            w = {k: v.detach().contiguous().float() for k, v in self.effective_weights().items()}
            n = h.shape[0]
            rows = n // x.shape[0]
            if rows * x.shape[0] != n:
                raise ValueError("h rows must be a multiple of x rows")
            f, _ = ops.dyn_eval(h.contiguous().float(), x.contiguous().float(), w, self.dyn_cfg(), rows_per_image=rows)
        return f

    def eval_dot(self, t, h_tuple, x):
        """classification.py:104-115."""
        return self._eval(h_tuple[0], x)

    def eval_dot_light(self, h, x):
        """classification.py:117-126."""
        return self._eval(h, x)

    def ode_forward(self, t, h_tuple):
        """classification.py:128-132."""
        assert self.static_state is not None, "[ERROR] You forgot to set static state before calling forward."
        return self.eval_dot(t, h_tuple, self.static_state)
