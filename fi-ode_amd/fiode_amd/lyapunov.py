"""LyapunovLearning with the fused HIP training step (pl_modules.py:338-502).

``LyapunovLossFn`` is the drop-in for the reference's per-sample autograd graph
(x_in expand -> sampler -> jvp(DecisionBoundary, eval_dot) -> relu -> mean, pl_modules.py:394-466):
one call of ``fiode_lyap_step`` computes the loss, the logging statistics and the gradient of the
loss w.r.t. the effective dynamics weights and the backbone features; backward() only scales the
saved gradients by the incoming grad and hands them to autograd, which continues through the
Cayley maps and the backbone.

pytorch_lightning and hydra are absent in this image, so ``LyapunovLearning`` is a plain
nn.Module keeping the LightningModule method names (training_step, compute_loss,
validation_step, configure_optimizers, log, current_epoch, global_step).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from . import ops
from .dynamics import OrthoClassDynProjectSimplexLips
from .models import IVP, DefaultOutputFun
from .odeint import make_solver_params
from .optim import FiodeAdam, FiodeAdamW
from .sampling import CompositeSampler, CompositeSamplerScheduler, TrajectorySampler
from .streams import new_stream


class LyapunovLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_feat, Q1, b1, Qx, bx, Q2, b2, Q3, b3, y, plan: dict):
        w = {"Q1": Q1, "b1": b1, "Qx": Qx, "bx": bx, "Q2": Q2, "b2": b2, "Q3": Q3, "b3": b3}
        w = {k: v.detach().contiguous() for k, v in w.items()}
        sc, grads, dbg = ops.lyap_step(
            x_feat.detach().contiguous(), y, w, plan["dyn"], sample_size=plan["S"], n_uniform=plan["S1"],
            sampler=plan["sampler"], dropout_mode=plan["dropout_mode"], kappa=plan["kappa"], seed=plan["seed"],
            offset=plan["offset"], h=plan.get("h"), masks=plan.get("masks"), debug=plan.get("debug", False),
            out=plan.get("out"), offset_dev=plan.get("offset_dev"), kappa_dev=plan.get("kappa_dev"))
        plan["scalars"] = sc
        plan["debug_out"] = dbg
        g = [grads[k] for k in ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")]
        ctx.save_for_backward(*g)
        return sc[0].clone()

    @staticmethod
    def backward(ctx, go):
        g = ctx.saved_tensors
        # the upstream scale on all nine gradients in one multi-tensor launch (was nine multiplies
        # between the solve's forward and backward on the step stream); same float32 products
        return tuple(torch._foreach_mul(list(g), go)) + (None, None)


class ODETrainFn(torch.autograd.Function):
    """y_hat = odeint(h_dot, h0, [0, t_max], method='rk4') in train mode, differentiable
    (fiode_odetrain_forward / _backward); the train_ode branch of pl_modules.py:490-493."""

    @staticmethod
    def forward(ctx, x_feat, Q1, b1, Qx, bx, Q2, b2, Q3, b3, h0, plan: dict):
        w = {"Q1": Q1, "b1": b1, "Qx": Qx, "bx": bx, "Q2": Q2, "b2": b2, "Q3": Q3, "b3": b3}
        w = {k: v.detach().contiguous() for k, v in w.items()}
        xf = x_feat.detach().contiguous()
        y, stats, ws = ops.odetrain_forward(xf, h0.detach().float().contiguous(), w, plan["dyn"], plan["cfg"],
                                            masks=plan.get("masks"), offset_dev=plan.get("offset_dev"))
        plan["stats"] = stats
        plan["status_word"] = ops.odetrain_status_word(ws, plan["cfg"])
        ctx.plan, ctx.w, ctx.xf, ctx.ws = plan, w, xf, ws
        from . import cayley as _cy
        ctx.step_stream = _cy.STEP_STREAM
        return y

    @staticmethod
    def backward(ctx, g_y):
        # The forward ran on a side stream beside the fan-out kernels; the backward has nothing to
        # overlap with (the backbone backward needs its dL/dx_feat), so it runs on the step stream
        # that produces g_y and consumes the gradients (ODE_BWD_ON_MAIN: no cross-queue hops).
        from . import cayley as _cy

        def run():
            grads, _ = ops.odetrain_backward(g_y.contiguous(), ctx.xf, ctx.w, ctx.plan["dyn"], ctx.plan["cfg"],
                                             ctx.ws)
            return tuple(grads[k] for k in ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3"))
        out = _cy._run_on_step_stream(ODE_BWD_ON_MAIN, ctx.step_stream, run)
        ctx.ws = None
        return tuple(out) + (None, None)


ODE_BWD_ON_MAIN = True


class ODENllFn(torch.autograd.Function):
    """F.nll_loss(torch.log(y_hat), y) as one kernel forward (fiode_ode_nll, which also writes
    d loss / d y_hat) and one multiply backward -- the train_ode loss term between the solve's
    forward and backward kernels, which sits on the step's critical path (pl_modules.py:494-497)."""

    @staticmethod
    def forward(ctx, y_hat, y):
        yh = y_hat.detach().contiguous().float()
        B = yh.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=yh.device)
        gunit = torch.empty_like(yh)
        L.check(L.lib().fiode_ode_nll(ops._stream(yh.device), B, yh.data_ptr(), y.contiguous().data_ptr(),
                                      loss.data_ptr(), gunit.data_ptr()), "fiode_ode_nll")
        ctx.save_for_backward(gunit)
        return loss

    @staticmethod
    def backward(ctx, go):
        gunit, = ctx.saved_tensors
        return gunit * go, None


class ODELossMixFn(torch.autograd.Function):
    """loss * (1 - p) + F.nll_loss(torch.log(y_hat), y) * p (pl_modules.py:494-500) as ONE kernel
    forward (fiode_ode_loss_mix, which also writes p * d nll / d y_hat) and two multiplies backward,
    so the solve's backward starts one kernel after its forward.  Returns (total, loss_ode); the
    second output is for logging (no gradient)."""

    @staticmethod
    def forward(ctx, loss, y_hat, y, p: float):
        yh = y_hat.detach().contiguous().float()
        B = yh.shape[0]
        lo = loss.detach().reshape(1).contiguous().float()
        total = torch.empty((), dtype=torch.float32, device=yh.device)
        loss_ode = torch.empty((), dtype=torch.float32, device=yh.device)
        gunit = torch.empty_like(yh)
        L.check(L.lib().fiode_ode_loss_mix(ops._stream(yh.device), B, yh.data_ptr(), y.contiguous().data_ptr(),
                                           lo.data_ptr(), float(p), loss_ode.data_ptr(), total.data_ptr(),
                                           gunit.data_ptr()), "fiode_ode_loss_mix")
        ctx.save_for_backward(gunit)
        ctx.p = float(p)
        ctx.mark_non_differentiable(loss_ode)
        return total, loss_ode

    @staticmethod
    def backward(ctx, go, _g_ode):
        gunit, = ctx.saved_tensors
        return go * (1.0 - ctx.p), gunit * go, None, None


# attribute GraphTrainStep sets on the gradient seed it passes to backward(): a float32 scalar 1.0
UNIT_GRAD = "_fiode_unit_grad"

# The dynamics weights' gradient of the training loss as its own autograd node on a side stream
# (_DynWeightTapFn): LyapODELossFn's backward then ends with dL/dx_feat, which alone the backbone's
# backward waits for
DYN_WGRAD_SIDE = os.environ.get("FIODE_DYN_WGRAD_SIDE", "1") != "0"


_ONES: dict = {}


def _one(dev) -> torch.Tensor:
    t = _ONES.get(str(dev))
    if t is None:
        t = _ONES[str(dev)] = torch.ones(1, dtype=torch.float32, device=dev)
    return t


class _DynWeightTapFn(torch.autograd.Function):
    """Carries the dynamics weights' gradients of LyapODELossFn to the weights.  Its forward (applied
    on a side stream) returns a token that LyapODELossFn takes as an input; LyapODELossFn's backward
    returns the token's gradient after the solve's adjoint sweep and dL/dx_feat, and leaves the
    weight-gradient work (the solve's weight-gradient chain, the fan-out's saved weight gradients
    added) in ``box``.  Autograd runs this node's backward after it, on the side stream its forward
    ran on, and synchronises the streams itself -- so the backbone's backward (on the step's stream)
    starts right after dL/dx_feat instead of after the weight-gradient chain."""

    @staticmethod
    def forward(ctx, box: dict, *weights):
        ctx.box = box
        return torch.empty((), dtype=torch.float32, device=weights[0].device)

    @staticmethod
    def backward(ctx, _gtok):
        fn = ctx.box.pop("weights")
        ctx.box = None
        return (None,) + tuple(fn())


class LyapODELossFn(torch.autograd.Function):
    """The configs[1] training loss as ONE autograd node (pl_modules.py:444-500): the fused
    Lyapunov step, the train_ode RK4 solve (launched first on ``ode_stream`` when given, so it
    overlaps the fan-out kernels), the nll term and the mix  loss * (1 - p) + nll(log y_hat) * p.
    Backward: the solve's backward with dL/dy_hat = go * p * d nll / d y_hat (the mix kernel's unit
    gradient), then its nine gradients plus the fused step's saved ones scaled by go * (1 - p), in
    one multi-tensor add.  (As three nodes, autograd inserted two scale kernels, a zero fill and
    one add kernel per shared input -- nine -- on the step's critical path.)  x_ode: the solve's
    features when they are not x_feat (ode_reuse_features False), else None."""

    @staticmethod
    def forward(ctx, x_feat, x_ode, Q1, b1, Qx, bx, Q2, b2, Q3, b3, h0, y, plan: dict, oplan: dict, p: float,
                ode_stream, box=None, tok=None):
        from .cayley import _prefetch, _take
        w = {"Q1": Q1, "b1": b1, "Qx": Qx, "bx": bx, "Q2": Q2, "b2": b2, "Q3": Q3, "b3": b3}
        w = {k: v.detach().contiguous() for k, v in w.items()}
        xf = x_feat.detach().float().contiguous()
        xo = xf if x_ode is None else x_ode.detach().float().contiguous()

        def solve():
            return ops.odetrain_forward(xo, h0.detach().float().contiguous(), w, oplan["dyn"], oplan["cfg"],
                                        masks=oplan.get("masks"), offset_dev=oplan.get("offset_dev"))
        pre = _prefetch(ode_stream, solve) if ode_stream is not None else None
        res = None if pre is not None else solve()
        sc, grads, dbg = ops.lyap_step(
            xf, y, w, plan["dyn"], sample_size=plan["S"], n_uniform=plan["S1"],
            sampler=plan["sampler"], dropout_mode=plan["dropout_mode"], kappa=plan["kappa"], seed=plan["seed"],
            offset=plan["offset"], h=plan.get("h"), masks=plan.get("masks"), debug=plan.get("debug", False),
            out=plan.get("out"), offset_dev=plan.get("offset_dev"), kappa_dev=plan.get("kappa_dev"))
        plan["scalars"] = sc
        plan["debug_out"] = dbg
        ctx.lyap = [grads[k] for k in ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")]
        # lyap * (1 - p) for a unit seed (GraphTrainStep), made here on the fan-out's stream before
        # it joins the solve: this multi-tensor kernel runs beside the solve instead of after its
        # backward (on the captured step's critical path)
        ctx.lyap_unit = torch._foreach_mul(ctx.lyap, 1.0 - float(p))
        if pre is not None:
            main = torch.cuda.current_stream(xf.device)
            main.wait_event(pre[1])
            for t in pre[0]:
                t.record_stream(main)
            res = pre[0]
        y_hat, stats, ws = res
        oplan["stats"] = stats
        oplan["status_word"] = ops.odetrain_status_word(ws, oplan["cfg"])
        B = y_hat.shape[0]
        total = torch.empty((), dtype=torch.float32, device=y_hat.device)
        loss_ode = torch.empty((), dtype=torch.float32, device=y_hat.device)
        gunit = torch.empty_like(y_hat)
        L.check(L.lib().fiode_ode_loss_mix(ops._stream(y_hat.device), B, y_hat.data_ptr(), y.contiguous().data_ptr(),
                                           sc.data_ptr(), float(p), loss_ode.data_ptr(), total.data_ptr(),
                                           gunit.data_ptr()), "fiode_ode_loss_mix")
        plan["loss_ode"] = loss_ode
        plan["y_hat"] = y_hat
        ctx.ode = (gunit, xo, w, oplan, ws)
        ctx.p = float(p)
        ctx.split = x_ode is not None
        ctx.box = box
        return total

    @staticmethod
    def backward(ctx, go):
        # ode + lyap * ((1 - p) go), summed as autograd's three-node graph sums it (bit for bit,
        # tests/test_gpu_odetrain.py); when go is GraphTrainStep's unit seed (``UNIT_GRAD``, exactly
        # 1.0) the products by go are exact and skipped, and (1 - p) is a host scalar: on the captured
        # step's critical path that drops three small kernels (the seed's ones fill, gunit * go,
        # go * (1 - p)) in front of / behind the solve's backward
        gunit, xo, w, oplan, ws = ctx.ode
        ctx.ode = None
        unit = getattr(go, UNIT_GRAD, False)
        g_y = gunit if unit else gunit * go
        box, ctx.box = ctx.box, None
        if box is not None:
            # dL/dx_feat here (the adjoint sweep); the weights' gradients in _DynWeightTapFn's backward
            lyap = ctx.lyap_unit if unit else torch._foreach_mul(ctx.lyap, go * (1.0 - ctx.p))
            ctx.lyap = ctx.lyap_unit = None
            if ctx.split:
                gxo = ops.odetrain_backward_x(g_y, xo, w, oplan["dyn"], oplan["cfg"], ws)
                gx = lyap[0]
            else:      # ode + lyap inside the dL/dx_feat kernel (times an exact 1.0: the same sum)
                gx = ops.odetrain_backward_x(g_y, xo, w, oplan["dyn"], oplan["cfg"], ws, gx_add=lyap[0],
                                             gx_add_scale=_one(g_y.device))
                gxo = None

            def weights():       # (on the tap's side stream: what it reads was allocated elsewhere)
                side = torch.cuda.current_stream(xo.device)
                for t in [xo, ws] + list(w.values()) + list(lyap[1:]):
                    t.record_stream(side)
                gr = ops.odetrain_backward_weights(xo, w, oplan["dyn"], oplan["cfg"], ws)
                ode = [gr[k] for k in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")]
                torch._foreach_add_(ode, lyap[1:])
                return ode
            box["weights"] = weights
            tg = go if go.dim() == 0 else go.reshape(())
            return (gx, gxo) + (None,) * 8 + (None, None, None, None, None, None, None, tg)
        gr, _ = ops.odetrain_backward(g_y, xo, w, oplan["dyn"], oplan["cfg"], ws)
        keys = ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")
        ode = [gr[k] for k in keys]
        lyap = ctx.lyap_unit if unit else torch._foreach_mul(ctx.lyap, go * (1.0 - ctx.p))
        ctx.lyap = ctx.lyap_unit = None
        if ctx.split:     # the solve's features are another tensor: its gradient goes there
            torch._foreach_add_(ode[1:], lyap[1:])
            gx, gxo = lyap[0], ode[0]
        else:
            torch._foreach_add_(ode, lyap)
            gx, gxo = ode[0], None
        return (gx, gxo) + tuple(ode[1:]) + (None, None, None, None, None, None, None, None)


class DecisionBoundary(nn.Module):
    """lya_cands.py:72-94 (kept for the validation/ODE path; the training step fuses it)."""

    def __init__(self, on_simplex=False, log_mode=False, num_class=10):
        super().__init__()
        self.on_simplex, self.log_mode, self.num_class = on_simplex, log_mode, num_class

    def forward(self, state_output, y):
        prob = state_output if self.on_simplex else F.softmax(state_output, dim=1)
        prob_y = torch.gather(prob, 1, y[:, None])[:, 0]
        wrong = torch.masked_select(prob, ~F.one_hot(y, self.num_class).bool()).unflatten(
            0, (prob.shape[0], prob.shape[1] - 1))
        v = 1 + wrong.max(dim=-1).values - prob_y
        return torch.log(v) if self.log_mode else v


# the solve's h0 kept contiguous between steps (tools/ab_step.py `h0_copy`: copied every step)
H0_CACHE = True


class UniformInitFun(nn.Module):
    """dynamics/init_coordinates.py:38-44: h0 = 1/C, static = param_map(x)."""

    def __init__(self, h_dims=(10,), param_map: Optional[nn.Module] = None):
        super().__init__()
        self.h_dims = tuple(h_dims)
        self.param_map = param_map if param_map is not None else nn.Identity()
        for i, d in enumerate(self.h_dims):
            self.register_buffer(f"h0_{i}", torch.ones(d) / d)

    def forward(self, x, dyn=None):
        # h0 as a broadcast view of the buffer (the reference's repeat is a copy kernel at the head of
        # the captured step's chain, and the fused training loss does not read it); an in-place write
        # into the view raises instead of touching the buffer
        h0 = tuple(getattr(self, f"h0_{i}")[None].expand(x.shape[0], -1).to(x.device) for i in range(len(self.h_dims)))
        return self.param_map(x), h0


class LyapunovLearning(nn.Module):
    """pl_modules.py:338-502 (order=1, act='relu', DecisionBoundary candidate)."""

    def __init__(self, order, h_sample_size, h_dist_lim, sampler: CompositeSampler,
                 sampler_scheduler: CompositeSamplerScheduler, dynamics: OrthoClassDynProjectSimplexLips,
                 init_fun: UniformInitFun, lya_cand=None, output=None, n_input=None, n_output=10, t_max=1.0,
                 train_ode_solver="dopri5", train_ode_tol=1e-6, val_ode_solver="dopri5", val_ode_tol=1e-6,
                 opt_name="SGD", lr=1e-3, momentum=0.9, weight_decay=1e-4, decay_epochs=(30, 60, 90),
                 beta1=0.9, beta2=0.999, scheduler_name="cos_anneal", max_epochs=200, warmup=20,
                 adv_train=False, eps=36 / 255, norm="L2", simplex=False, act="relu", fix_backbone=False,
                 val_adv=True, barrier_loss=False, lips_train=False, relax_exp_stable=False, scaleLeps=3.0,
                 train_ode=False, train_ode_epoch=100, epoch_off_scale=10, lips_warmup=0, seed=0):
        super().__init__()
        if order != 1:
            raise NotImplementedError("order=1 (the reference raises for order 0; higher orders are unused)")
        if act != "relu":
            raise NotImplementedError("act='relu' is the README configuration")
        if barrier_loss or lips_train or relax_exp_stable or adv_train:
            raise NotImplementedError("barrier_loss / lips_train / relax_exp_stable / adv_train are off "
                                      "in the north-star configuration and not fused")
        self.train_ode, self.train_ode_epoch = bool(train_ode), int(train_ode_epoch)
        self.order, self.h_sample_size, self.h_dist_lim = order, h_sample_size, h_dist_lim
        self.sampler, self.sampler_scheduler = sampler, sampler_scheduler
        # same module tree as the reference (state_dict keys model.dyn_fun.*, model.init_coordinates.*)
        self.model = IVP(n_input=n_input, n_output=n_output, dyn_fun=dynamics, init_coordinates=init_fun,
                         output_fun=output if output is not None else DefaultOutputFun(), ode_tol=train_ode_tol,
                         ts=torch.linspace(0, t_max, 2))
        self.lya_cand = lya_cand if lya_cand is not None else DecisionBoundary(on_simplex=True)
        self.t_max = t_max
        self.use_adjoint = False
        self.train_ode_solver, self.train_ode_tol = train_ode_solver, train_ode_tol
        self.val_ode_solver, self.val_ode_tol = val_ode_solver, val_ode_tol
        self.opt_name, self.lr, self.momentum, self.weight_decay = opt_name, lr, momentum, weight_decay
        self.fix_backbone = fix_backbone
        self.decay_epochs, self.betas = list(decay_epochs), (beta1, beta2)
        self.scheduler_name, self.max_epochs, self.warmup = scheduler_name, max_epochs, warmup
        self.simplex, self.act, self.eps, self.norm = simplex, act, eps, norm
        self.epoch_off_scale = epoch_off_scale
        self.current_epoch = 0
        self.global_step = 0
        self.seed = seed
        self._rng_offset = 0
        self.rng_counter: Optional[torch.Tensor] = None   # device step counter (graph replay)
        self.parallel_cayley = True     # Cayley maps of the step on side streams (training, ROCm)
        self.lyap_after_ode = False     # fan-out kernels start after the train_ode forward (see compute_loss)
        # train_ode branch: reuse the step's backbone features (True) or re-run the backbone as the
        # reference's self.model(x) does (False); DESIGN.md section 5 (common-subexpression reuse)
        self.ode_reuse_features = True
        # the configs[1] loss as one autograd node (LyapODELossFn); False: three nodes (the Lyapunov
        # step, the solve, the mix) as in round 1
        self.fused_ode_loss = True
        self._side_streams = None
        # capture points of the Cayley maps' prefetch (_prefetch_weights): the 4096 -> 512 map right
        # after the input kernels, the other maps after conv layer 2 (None: all of them at the input)
        self._prefetch_late_at = 2
        self.logged: Dict[str, float] = {}
        self._out = None

    @property
    def dyn_fun(self):
        return self.model.dyn_fun

    @property
    def init_coordinates(self):
        return self.model.init_coordinates

    @property
    def train_solver_params(self):
        return make_solver_params(self.train_ode_solver, self.train_ode_tol)

    @property
    def val_solver_params(self):
        return make_solver_params(self.val_ode_solver, self.val_ode_tol)

    def forward(self, x, t_steps=2, return_traj=False):
        """ODELearning.forward (pl_modules.py:322-325): validation/inference ODE solve."""
        return self.model(x, ts=torch.linspace(0.0, self.t_max, t_steps, device=x.device),
                          int_params=self.val_solver_params, use_adjoint=self.use_adjoint, return_traj=return_traj)

    def validation_step(self, batch, batch_idx=0):
        """GeneralLearning.validation_step without attacks (val_adv=False, pl_modules.py:203-219)."""
        x, y = batch
        with torch.no_grad():
            net_out = self(x)
        error = (net_out.argmax(dim=-1) != y).float().mean()
        if self.simplex:
            loss = F.nll_loss(torch.log(torch.clamp(net_out, min=1e-12)), y)
        else:
            loss = F.cross_entropy(net_out, y)
        # self.log(..., sync_dist=True) (pl_modules.py:217-219): the mean over ranks, all three
        # values in one all-reduce (distributed.MetricReducer); a single process logs its own
        from .distributed import MetricReducer
        import torch.distributed as dist
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if world > 1:
            red = MetricReducer(["validation_loss", "validation_error"], loss.device).reduce(
                {"validation_loss": loss, "validation_error": error}, world)
            self.log("validation_loss", red["validation_loss"])
            self.log("validation_error", red["validation_error"])
            self.log("validation_adv_error", red["validation_error"])
        else:
            self.log("validation_loss", loss)
            self.log("validation_error", error)
            self.log("validation_adv_error", error)
        return loss

    # Lightning-like surface -------------------------------------------------------------------
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict: bool = True, **kwargs):
        """LightningModule.load_from_checkpoint as the reference calls it (utils.py:14-28,
        robustness/eval_utils.py:92-107): build from the config kwargs, load ``state_dict``
        (torch.load(weights_only=True)), keep epoch / global_step of the file."""
        from .checkpoint import load_from_checkpoint
        mod = cls(**kwargs)
        info = load_from_checkpoint(mod, checkpoint_path, strict=strict, map_location=map_location)
        mod.loaded_checkpoint = info
        return mod

    def log(self, name, value, **kw):
        self.logged[name] = value

    def configure_optimizers(self, capturable: bool = False, fused: Optional[bool] = None):
        """pl_modules.py:97-147 (Adam/AdamW/SGD; cosine or step schedule; warm-up Adam).
        ``capturable``: Adam/AdamW keep their step counts on the device so the optimizer step
        can be captured in a hipGraph (fiode_amd.graph_step).  ``fused`` (default on ROCm device
        parameters): Adam/AdamW as fiode_amd.optim.FiodeAdam / FiodeAdamW -- torch's classes (same
        state and state_dict) whose step is one HIP launch over all parameters (adam.hip)."""
        params = list(self.parameters())
        if fused is None:
            fused = bool(params) and params[0].is_cuda
        fk = {"fused": True, "capturable": capturable} if fused else {"capturable": capturable}
        adam, adamw = (FiodeAdam, FiodeAdamW) if fused else (torch.optim.Adam, torch.optim.AdamW)
        if self.current_epoch < self.warmup:
            return [adam(params, lr=1e-3, weight_decay=5e-4, amsgrad=False, betas=self.betas, **fk)]
        if self.opt_name == "Adam":
            opt = adam(params, lr=self.lr, weight_decay=self.weight_decay, betas=self.betas, **fk)
        elif self.opt_name == "AdamW":
            opt = adamw(params, lr=self.lr, weight_decay=self.weight_decay, betas=self.betas, **fk)
        elif self.opt_name == "SGD":
            # fix_backbone: SGD over the dynamics' parameters only (pl_modules.py:110-114)
            sgd_params = list(self.model.dyn_fun.parameters()) if self.fix_backbone else params
            opt = torch.optim.SGD(sgd_params, lr=self.lr, momentum=self.momentum, weight_decay=self.weight_decay)
        else:
            raise RuntimeError(f"[ERROR] Invalid Optimizer Param: {self.opt_name}")
        if self.scheduler_name == "cos_anneal":
            sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=self.max_epochs)
        elif self.scheduler_name == "step":
            sch = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=self.decay_epochs, gamma=0.1)
        else:
            return [opt]
        return [opt], [sch]

    def training_step(self, batch, batch_idx=0):
        x, y = batch
        loss = self.compute_loss(x, y, x.shape[0], self.act)
        self.log("training_loss", loss)
        return loss

    # the hot path -----------------------------------------------------------------------------
    def current_kappa(self) -> float:
        """pl_modules.py:447-450."""
        dyn = self.dyn_fun
        if self.global_step < dyn.kappa_length:
            return self.global_step / dyn.kappa_length * dyn.kappa
        return dyn.kappa

    def kappa_device(self) -> Optional[torch.Tensor]:
        """The kappa ramp (pl_modules.py:447-448) on the device, for a captured step: with the
        anchor GraphTrainStep sets (global_step - rng_counter at capture), global_step = rng_counter +
        anchor is read from the device counter every replay advances; kappa = global_step /
        kappa_length * kappa in float64 (Python's arithmetic), rounded to float32 like torch's scalar
        operand, or kappa once global_step >= kappa_length.  None = the host value (eager steps)."""
        anchor = getattr(self, "_kappa_anchor", None)
        dyn = self.dyn_fun
        if anchor is None or self.rng_counter is None or not dyn.kappa_length:
            return None
        step = self.rng_counter.double() + float(anchor)
        L_ = float(dyn.kappa_length)
        return torch.where(step < L_, step / L_ * float(dyn.kappa),
                           torch.full_like(step, float(dyn.kappa))).float()

    def step_plan(self, y: torch.Tensor, h: Optional[torch.Tensor] = None, masks: Optional[torch.Tensor] = None,
                  debug: bool = False, static_state: Optional[torch.Tensor] = None) -> dict:
        mix = self.sampler_scheduler.get_mixer_coefficients(self.current_epoch)
        for i, m in enumerate(mix):
            self.log(f"mixing_weight_{i}", float(m))
        kind, s1 = self.sampler.kernel_plan(self.h_sample_size, mix)
        drop = L.FIODE_DROPOUT_PHILOX if self.training else L.FIODE_DROPOUT_OFF
        if masks is not None:
            drop = L.FIODE_DROPOUT_GIVEN
        if h is not None:
            kind = L.FIODE_SAMPLER_GIVEN
        elif kind == L.FIODE_SAMPLER_TRAJECTORY and s1 < self.h_sample_size:
            # TrajectorySampler rows (sampler.py:156-166): the solve's states, computed before the step
            traj = next(t for t in self.sampler.samplers if isinstance(t, TrajectorySampler))
            h = traj.trajectory(self, static_state, self.h_sample_size - s1)
        plan = dict(dyn=self.dyn_fun.dyn_cfg(), S=self.h_sample_size, S1=s1, sampler=kind, dropout_mode=drop,
                    kappa=self.current_kappa(), kappa_dev=self.kappa_device(), seed=self.seed,
                    offset=self._rng_offset if self.rng_counter is None else 0, h=h, masks=masks,
                    debug=debug, out=None, offset_dev=self.rng_counter)
        self._rng_offset += 1
        return plan

    def _prefetch_weights(self, device):
        """Launch every Cayley map of the step (backbone convs / linears, dynamics) on side streams:
        they depend only on the weights, and their inverses are latency-bound small kernels, so they
        overlap each other and the convolutions.  Layers join them when they reach them (autograd
        runs their backward on the same streams).

        Capture order: the hipGraph executor dispatches nodes in capture order over a few hardware
        queues, so maps captured ahead of the main stream's first kernels hold those kernels back.
        The launches are therefore captured by a hook on the backbone's conv stack: the 4096 -> 512
        map (the first one the step needs, and the longest chain) right after the step's input
        kernels, the other linear maps and the dynamics' maps after conv layer 2 (``_prefetch_late_at``;
        round 4: 1.476 -> 1.416 ms with both sides' captures picked from 4 placements,
        tools/ab_step.py), then the conv maps (conv maps computed one step ahead by GraphTrainStep
        skip their launch here).  Measured alternatives
        (deferral past conv layers, one stream per map, one chain for all
        linear maps, one batched inverse for both 512 x 512 systems) were all slower or equal."""
        if not getattr(self, "_in_input_hook", False):
            bb = self.init_coordinates.param_map
            target = bb[-1] if isinstance(bb, torch.nn.Sequential) else bb

            at = getattr(self, "_prefetch_at", -1)      # tools/ab_step.py probes later capture points

            late = getattr(self, "_prefetch_late_at", None)   # the maps after the first: after this conv layer

            last = max(x for x in (at, late) if x is not None)

            def hook(i, _t=target, _at=at):
                if i == _at or (late is not None and i == late):
                    self._in_input_hook = True
                    self._prefetch_part = None if late is None else ("first" if i == _at else "rest")
                    try:
                        self._prefetch_weights(device)
                    finally:
                        self._in_input_hook = False
                        self._prefetch_part = None
                if i >= last:
                    _t.after_conv_hook = None
            target.after_conv_hook = hook
            return
        if self._side_streams is None:
            self._side_streams = [new_stream(device) for _ in range(4)]
        s = self._side_streams
        convs, lins = [], []
        for m in self.init_coordinates.modules():
            if hasattr(m, "prefetch") and m is not self.dyn_fun:
                (convs if hasattr(m, "spectral_weight") else lins).append(m)
        order = getattr(self, "_map_streams", (1, 2, 3, 3))   # side stream of each linear map, then dyn's
        part = getattr(self, "_prefetch_part", None)
        nfirst = getattr(self, "_prefetch_first_lins", 1)       # linear maps in the first stage
        dyn_first = getattr(self, "_prefetch_dyn_first", False)
        for i, l in enumerate(lins):
            if part is None or (part == "first") == (i < nfirst):
                l.prefetch(s[order[min(i, 2)]])
        if part is None or (part == "first") == dyn_first:
            self.dyn_fun.prefetch(s[order[3]])
        if part != "rest":             # (before conv layer 0: a map prefetched later would go unused)
            for c in convs:
                c.prefetch(s[0])

    def compute_loss(self, x, y, batch_size=None, act="relu", h=None, masks=None, debug=False):
        """pl_modules.py:390-502 with the per-sample graph fused (LyapunovLossFn)."""
        from . import cayley as _cy
        step_stream = torch.cuda.current_stream(x.device) if x.is_cuda else None
        with _cy.step_stream_scope(step_stream):
            return self._compute_loss(x, y, h=h, masks=masks, debug=debug)

    def _compute_loss(self, x, y, h=None, masks=None, debug=False):
        if self.current_epoch == self.epoch_off_scale:
            self.dyn_fun.scale_nominal = False
        if self.parallel_cayley and self.training and x.is_cuda and self.dyn_fun.cayley:
            self._prefetch_weights(x.device)
        static_state, _ = self.init_coordinates(x, self.dyn_fun)
        bb = self.init_coordinates.param_map
        if isinstance(bb, torch.nn.Sequential) and getattr(bb[-1], "after_conv_hook", None) is not None:
            bb[-1].after_conv_hook = None       # never left armed for a later (e.g. validation) forward
        plan = self.step_plan(y, h=h, masks=masks, debug=debug, static_state=static_state)
        w = self.dyn_fun.effective_weights()
        ode_on = self.train_ode and self.current_epoch > self.train_ode_epoch
        if (ode_on and self.fused_ode_loss and static_state.is_cuda and self.simplex and y.dtype == torch.int64
                and not self.lyap_after_ode):
            return self._lyap_ode_loss(x, static_state, w, y, plan)
        if ode_on:        # launched first: on ROCm it runs on a side stream beside the fan-out kernels
            feat_ode = static_state
            if not self.ode_reuse_features:
                # reference order: self.model(x, ...) re-runs the backbone (pl_modules.py:491); the
                # default reuses the features (the backbone is deterministic: same value, one pass)
                feat_ode, _ = self.init_coordinates(x, self.dyn_fun)
            y_hat = self._ode_launch(feat_ode.float(), w)
            if isinstance(y_hat, tuple) and self.lyap_after_ode:
                # k_ot_fwd is a persistent latency chain whose 8 workgroups exchange QP exit masks:
                # dispatched beside the fan-out kernels, some of its workgroups wait for CUs while the
                # resident ones spin.  Ordering the fan-out after the solve's forward lets the solve
                # run alone and the fan-out overlap its backward (measured: -0.2 ms per step).
                torch.cuda.current_stream(static_state.device).wait_event(y_hat[1])
        loss = LyapunovLossFn.apply(static_state.float(), w["Q1"], w["b1"], w["Qx"], w["bx"], w["Q2"], w["b2"],
                                    w["Q3"], w["b3"], y, plan)
        sc = plan["scalars"]
        self.log("kappa", plan["kappa_dev"] if plan.get("kappa_dev") is not None else plan["kappa"])
        self.log("effective_batch_size", sc[1])
        self.log("mean_active_constraints", sc[2])
        self.last_plan = plan
        if ode_on:
            return self._ode_loss(loss, y_hat, y)
        return loss

    def status_words(self) -> list:
        """Device int32 [1] status words of the last train_ode solve (forward stats[3]; the dopri5
        solve's forward + backward word): what a step guard reads (optim.StepGuard)."""
        plan = getattr(self, "last_ode_plan", None)
        if not plan or not (self.train_ode and self.current_epoch > self.train_ode_epoch):
            return []
        return [t for t in (plan["stats"][3:4] if plan.get("stats") is not None else None,
                            plan.get("status_word")) if t is not None]

    def device_status(self) -> int:
        """Status of the last train_ode solve: 0 ok, 2 = the dopri5 attempt capacity was exhausted,
        3 = dt underflow, 4 = a workgroup's cross-workgroup exchange timed out (its outputs were
        poisoned with NaN).  One host read: call it every few hundred steps or at the epoch end."""
        return max([int(t[0]) for t in self.status_words()] or [0])

    def check_device_status(self) -> None:
        status = self.device_status()
        if status:
            what = {2: "the dopri5 attempt capacity (train_ode_max_attempts) was exhausted",
                    3: "dt underflow"}.get(status, "a cross-workgroup exchange timed out")
            raise RuntimeError(f"train_ode solve failed (status {status}: {what}); the step's loss is NaN")

    def ode_plan(self, batch: int, masks: Optional[torch.Tensor] = None) -> dict:
        """Solver plan of the train_ode solve (make_solver_params(train_ode_solver, train_ode_tol),
        pl_modules.py:24-35): 'rk4' with options.step_size = tol, or 'dopri5' with rtol = atol = tol
        (cifar_train.yaml:30,32), at most ``ode_attempt_capacity(batch)`` adaptive step attempts (the eval
        capacity of the device solve: ``train_ode_max_attempts`` or what 4 GiB of workspace holds;
        torchdiffeq has no cap -- more attempts report status 2 and a NaN loss, which the step guard
        keeps away from the parameters; see check_device_status)."""
        if self.use_adjoint:
            raise NotImplementedError("odeint_adjoint (SURVEY.md section 8f row 3)")
        if self.train_ode_solver not in ("rk4", "dopri5"):
            raise NotImplementedError(f"train_ode with {self.train_ode_solver!r}: the differentiable HIP solves are "
                                      "'rk4' and 'dopri5'")
        mode = L.FIODE_DROPOUT_PHILOX if self.training else L.FIODE_DROPOUT_OFF
        if masks is not None:
            mode = L.FIODE_DROPOUT_GIVEN
        sp = make_solver_params(self.train_ode_solver, self.train_ode_tol)
        off = self._rng_offset if self.rng_counter is None else 0
        if self.train_ode_solver == "rk4":
            cfg = ops.odetrain_config(batch, 0.0, float(self.t_max), float(sp["options"]["step_size"]), mode,
                                      seed=self.seed, offset=off)
        else:
            cfg = ops.odetrain_config(batch, 0.0, float(self.t_max), 0.0, mode, seed=self.seed, offset=off,
                                      method="dopri5", rtol=float(sp["rtol"]), atol=float(sp["atol"]),
                                      max_attempts=self.ode_attempt_capacity(batch))
        return dict(dyn=self.dyn_fun.dyn_cfg(), cfg=cfg, masks=masks, offset_dev=self.rng_counter)

    def ode_attempt_capacity(self, batch: int) -> int:
        """``train_ode_max_attempts`` if set, else the capacity 4 GiB of workspace holds
        (ops.odetrain_default_attempts; cached per batch size)."""
        cap = getattr(self, "train_ode_max_attempts", None)
        if cap:
            return int(cap)
        cache = self.__dict__.setdefault("_attempt_cap", {})
        if batch not in cache:
            cache[batch] = ops.odetrain_default_attempts(batch)
        return cache[batch]

    def _ode_launch(self, static_state, w, masks=None):
        """The train_ode solve (pl_modules.py:490-493).  The reference re-runs the backbone inside
        self.model(x); the backbone is deterministic (no dropout / batch norm), so static_state is
        reused.  Its persistent kernel occupies B/32 CUs for the whole solve, so on ROCm it is
        launched on a side stream and overlaps the fan-out kernels."""
        h0 = self._h0(static_state.shape[0])
        plan = self.ode_plan(static_state.shape[0], masks)
        # leaf parameters (the biases) enter the side-stream solve through views taken here, on the
        # step stream: their AccumulateGrad nodes then receive every gradient on the step stream
        # (a leaf used directly on two streams gets gradients from both: torch warns that this can
        # break graph capture)
        w = {k: (v.view_as(v) if v.is_leaf and v.requires_grad else v) for k, v in w.items()}
        args = (static_state, w["Q1"], w["b1"], w["Qx"], w["bx"], w["Q2"], w["b2"], w["Q3"], w["b3"], h0, plan)
        self.last_ode_plan = plan
        if static_state.is_cuda and self.parallel_cayley and getattr(self, "ode_side_stream", True):
            from .cayley import _prefetch
            if getattr(self, "_ode_stream", None) is None:
                self._ode_stream = new_stream(static_state.device, priority=getattr(self, "_ode_prio", -1))
            return _prefetch(self._ode_stream, lambda: ODETrainFn.apply(*args))
        return ODETrainFn.apply(*args)

    def _h0(self, B: int) -> torch.Tensor:
        """The solve's initial state h0 = 1/C for every row (init_coordinates.py:38-44) as the
        contiguous [B][C] the kernels read.  Kept from an eager call (the GraphTrainStep warm-up)
        while the buffer is unchanged, so a captured step holds no copy kernel right before the
        solve; never made inside a capture (a captured copy would only run at replay)."""
        h0_0 = self.init_coordinates.h0_0
        key = (B, h0_0.device, h0_0.data_ptr(), h0_0._version)
        c = getattr(self, "_h0_cache", None)
        if H0_CACHE and c is not None and c[0] == key:
            return c[1]
        h0 = h0_0[None].expand(B, -1).float().contiguous()
        if H0_CACHE and not (h0.is_cuda and torch.cuda.is_current_stream_capturing()):
            self._h0_cache = (key, h0)
        return h0

    def _lyap_ode_loss(self, x, static_state, w, y, plan):
        """The fused configs[1] loss (LyapODELossFn): one autograd node for the Lyapunov step, the
        train_ode solve and the mix (pl_modules.py:444-500)."""
        x_ode = None
        if not self.ode_reuse_features:
            # reference order: self.model(x, ...) re-runs the backbone (pl_modules.py:491)
            x_ode, _ = self.init_coordinates(x, self.dyn_fun)
        h0 = self._h0(static_state.shape[0])
        oplan = self.ode_plan(static_state.shape[0])
        self.last_ode_plan = oplan
        stream = None
        if self.parallel_cayley and getattr(self, "ode_side_stream", True):
            if getattr(self, "_ode_stream", None) is None:
                self._ode_stream = new_stream(static_state.device, priority=getattr(self, "_ode_prio", -1))
            stream = self._ode_stream
        p = min(0.98, (self.current_epoch - self.train_ode_epoch) / 50.0)
        keys = ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")
        if DYN_WGRAD_SIDE and static_state.is_cuda and torch.is_grad_enabled():
            box = {}
            if getattr(self, "_wtap_stream", None) is None:
                self._wtap_stream = new_stream(static_state.device)
            side, main = self._wtap_stream, torch.cuda.current_stream(static_state.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                tok = _DynWeightTapFn.apply(box, *[w[k] for k in keys])
            main.wait_stream(side)
            wd = [w[k].detach() for k in keys]
            total = LyapODELossFn.apply(static_state, x_ode, *wd, h0, y, plan, oplan, p, stream, box, tok)
        else:
            total = LyapODELossFn.apply(static_state, x_ode, *[w[k] for k in keys], h0, y, plan, oplan, p, stream)
        sc = plan["scalars"]
        self.log("kappa", plan["kappa_dev"] if plan.get("kappa_dev") is not None else plan["kappa"])
        self.log("effective_batch_size", sc[1])
        self.log("mean_active_constraints", sc[2])
        self.log("loss_ode", plan["loss_ode"])
        self.last_plan = plan
        return total

    def _ode_loss(self, loss, y_hat, y):
        """pl_modules.py:494-500: loss * (1 - p) + nll(log y_hat) * p."""
        if isinstance(y_hat, tuple):
            from .cayley import _take
            y_hat = _take(y_hat)
        p = min(0.98, (self.current_epoch - self.train_ode_epoch) / 50.0)
        if (self.simplex and y_hat.is_cuda and y.dtype == torch.int64 and y_hat.dim() == 2 and y_hat.shape[1] == 10
                and loss.is_cuda):
            total, loss_ode = ODELossMixFn.apply(loss, y_hat, y, p)
            self.log("loss_ode", loss_ode)
            return total
        if self.simplex:
            loss_ode = F.nll_loss(torch.log(y_hat), y)
        else:
            loss_ode = F.cross_entropy(y_hat, y)
        self.log("loss_ode", loss_ode)
        return loss * (1.0 - p) + loss_ode * p
