"""Data-parallel plumbing for the train step and certification (one process per GPU).

The reference trains under Lightning DDP (train_classification.py: ``pl.Trainer(gpus=..,
strategy=DDP)``, ``self.log(..., sync_dist=True)`` in pl_modules.py:480-484): every rank runs the
whole fan-out on its own images, DDP all-reduces the gradients (bucketed, 25 MB) and Lightning
reduces each logged scalar with its own collective.  The path has one real exchange step (the
gradient mean) and one bookkeeping exchange (the logged means), so here:

* ``GradAllReducer``  -- one persistent flat fp32 buffer holding every trainable gradient
  (~2.6 M floats = 10.5 MB for the README model), laid out in the order the backward finalises
  the gradients and all-reduced in a few contiguous buckets -- inside the captured step, each as
  soon as its gradients are final, overlapping the rest of the backward (DDP's bucketing); the
  views of ``p.grad`` point INTO the buffer, so no pack/unpack copies are made.
* ``MetricReducer``   -- the logged scalars of a step packed into one small tensor, one
  all-reduce (SUM, divided by world) instead of one collective per ``self.log``.
* ``shard_range``     -- contiguous image shards for certification / validation (no collective
  on the data path; one count all-reduce at the end, certify.allreduce_counts).

Everything works with the ``nccl`` (= RCCL on ROCm) backend on GPU ranks and ``gloo`` on CPU ranks
(tests/test_distributed.py runs world_size 2 over gloo).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist


def world_info():
    """(rank, world, local_rank) from the torch.distributed.run environment (defaults: 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(device_type: str = "cuda"):
    """Initialise the default group from env:// (nccl for GPU ranks, gloo for CPU); returns world."""
    rank, world, local = world_info()
    if world > 1 and not dist.is_initialized():
        backend = "nccl" if device_type == "cuda" else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, init_method="env://")
    return world


def shard_range(n: int, rank: int, world: int) -> range:
    """Contiguous shard [lo, hi) of n units for `rank` (ceil split; trailing ranks may be empty)."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return range(lo, min(n, lo + per))


class GradAllReducer:
    """Mean of the gradients over ranks from one persistent flat bucket, all-reduced in a few
    contiguous BUCKETS that follow the order in which the backward finalises the gradients (DDP's
    bucketing, sl_pipeline.py:157-170 via Lightning's DDP strategy).

    ``p.grad`` of every parameter is a view into ``self.flat``.  Two ways to run the collective:

    * ``allreduce()`` -- after the backward (eager, between graph replays; any backend): one
      all-reduce per bucket, then the 1/world scale;
    * ``arm(world, stream)`` before the backward and ``finish()`` after it -- a post-accumulate
      hook per parameter moves each fresh gradient into its bucket view and, once a bucket's last
      parameter has its gradient, launches that bucket's all-reduce on ``stream`` (ordered after the
      producing stream), so the collective of the early buckets runs while the rest of the backward
      does; ``finish()`` launches what is left and joins.  Used by GraphTrainStep with RCCL, where
      the whole step (collectives included) is one captured graph.

    The bucket layout comes from ``plan_buckets(order, cap_bytes)``: ``order`` = the parameters in
    the order their gradients became final in a warm-up backward (``record_order``), the flat
    bucket laid out in that order and cut into buckets of about ``cap_bytes``.  Until then: one
    bucket in ``params`` order.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("GradAllReducer: no trainable parameters")
        dev = self.params[0].device
        dtypes = {p.dtype for p in self.params}
        if len(dtypes) != 1:
            raise ValueError(f"GradAllReducer: mixed parameter dtypes {dtypes}")
        self.group = group
        self.numel = sum(p.numel() for p in self.params)
        # one float past the gradients: the step-guard slot (this rank's skip verdict, written just
        # before the last bucket's all-reduce; summed with the gradients, so any rank's bad step --
        # failed solve, non-finite loss -- makes every rank skip the optimizer step together)
        self.flat = torch.zeros(self.numel + 1, dtype=self.params[0].dtype, device=dev)
        self.guard_slot = self.flat[self.numel:]
        self.guard_writer = None          # callable(slot): launches the verdict kernel, or None
        self._hooks = []
        self._armed = None
        self._order_log = None
        self._layout(list(self.params), [len(self.params)])
        for p, v in zip(self.params, self.views):
            if p.grad is not None:
                v.copy_(p.grad)
            p.grad = v

    # ---- layout ------------------------------------------------------------------------------
    def _layout(self, order, cuts):
        """Flat bucket in ``order``; bucket k = parameters order[cuts[k-1]:cuts[k]]."""
        self.order = order
        self.views = [None] * len(self.params)
        pos = {id(p): i for i, p in enumerate(self.params)}
        o = 0
        starts = []
        for p in order:
            starts.append(o)
            self.views[pos[id(p)]] = self.flat[o:o + p.numel()].view_as(p)
            o += p.numel()
        self.buckets = []                 # (lo, hi) flat ranges; members as positions in params
        self.members = []
        lo_i = 0
        for c in cuts:
            lo = starts[lo_i]
            hi = starts[c] if c < len(order) else self.numel + 1     # the last bucket carries the slot
            self.buckets.append((lo, hi))
            self.members.append([pos[id(p)] for p in order[lo_i:c]])
            lo_i = c
        self.bucket_of = [0] * len(self.params)
        for k, m in enumerate(self.members):
            for i in m:
                self.bucket_of[i] = k

    def plan_buckets(self, order: Sequence[torch.nn.Parameter], cap_bytes: int = 4 << 20):
        """Lay the bucket out in ``order`` (gradients' ready order) and cut it every ~cap_bytes
        (a parameter never straddles two buckets)."""
        seen = {id(p) for p in order}
        order = list(order) + [p for p in self.params if id(p) not in seen]
        cuts, acc = [], 0
        for i, p in enumerate(order):
            acc += p.numel() * p.element_size()
            if acc >= cap_bytes and i + 1 < len(order):
                cuts.append(i + 1)
                acc = 0
        cuts.append(len(order))
        grads = [p.grad.detach().clone() if p.grad is not None else None for p in self.params]
        self._layout(order, cuts)
        for p, v, g in zip(self.params, self.views, grads):
            if g is not None:
                v.copy_(g)
            else:
                v.zero_()
            p.grad = v

    def record_order(self):
        """Start logging the order in which the next backward finalises the gradients."""
        self._order_log = []
        if not self._hooks:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(lambda _p, i=i: self._on_grad(i)))

    def recorded_order(self) -> List[torch.nn.Parameter]:
        log, self._order_log = self._order_log or [], None
        return [self.params[i] for i in log]

    # ---- collectives ------------------------------------------------------------------------------
    def rebind(self):
        """Re-point grads into the bucket (after something replaced p.grad, e.g. set_to_none)."""
        for p, v in zip(self.params, self.views):
            if p.grad is None:
                v.zero_()
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
            p.grad = v

    def zero_grad(self):
        self.flat.zero_()

    def gather(self):
        """Move the gradients autograd just produced (fresh tensors: the backward ran with p.grad =
        None, so AccumulateGrad stole its results instead of adding them into the bucket one kernel
        per parameter) into the bucket with ONE multi-tensor copy, and re-point p.grad at the bucket
        views.  A parameter that received no gradient gets zeros."""
        have = [(v, p.grad) for v, p in zip(self.views, self.params) if p.grad is not None]
        if have:
            torch._foreach_copy_([v for v, _ in have], [g for _, g in have])
        for v, p in zip(self.views, self.params):
            if p.grad is None:
                v.zero_()
            p.grad = v
        return self.flat[:self.numel]

    def allreduce(self, world: Optional[int] = None, force: bool = False):
        world = dist.get_world_size(self.group) if world is None else world
        if world > 1 or force:
            self.rebind()
            if self.guard_writer is not None:
                self.guard_writer(self.guard_slot)
            for lo, hi in self.buckets:
                dist.all_reduce(self.flat[lo:hi], group=self.group)
            self.flat.div_(world)
        return self.flat[:self.numel]

    def arm(self, world: int, stream: torch.cuda.Stream, force: bool = False):
        """Overlapped all-reduce of the next backward (see the class docstring).  The backward must
        run with p.grad = None (GraphTrainStep does)."""
        if not self._hooks:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(lambda _p, i=i: self._on_grad(i)))
        self._armed = dict(world=world, stream=stream, force=force, left=[len(m) for m in self.members],
                           fresh=[None] * len(self.params), done=[False] * len(self.buckets), keep=[])

    def _on_grad(self, i):
        if self._order_log is not None:
            self._order_log.append(i)
        st = self._armed
        if st is None:
            return
        # the gradient was produced on the hook's current stream (autograd runs a node on its
        # forward's stream, side streams included): the comm stream waits for every one of them
        st["stream"].wait_stream(torch.cuda.current_stream(st["stream"].device))
        k = self.bucket_of[i]
        p = self.params[i]
        st["fresh"][i] = p.grad
        st["left"][k] -= 1
        if st["left"][k] == 0:
            self._launch(k)

    def _launch(self, k):
        st = self._armed
        comm = st["stream"]
        comm.wait_stream(torch.cuda.current_stream(comm.device))
        with torch.cuda.stream(comm):
            pairs = []
            for i in self.members[k]:
                g = st["fresh"][i]
                v = self.views[i]
                if g is None:
                    v.zero_()
                elif g.data_ptr() != v.data_ptr():
                    pairs.append((v, g))
                    g.record_stream(comm)         # read on the comm stream: no reuse before that
                    st["keep"].append(g)
                self.params[i].grad = v
            if pairs:
                torch._foreach_copy_([v for v, _ in pairs], [g for _, g in pairs])
            if k == len(self.buckets) - 1 and self.guard_writer is not None:
                # the last bucket's gradients are final, so everything upstream of them (the loss,
                # the train_ode solve forward and backward) has run: its verdict is final too
                self.guard_writer(self.guard_slot)
            lo, hi = self.buckets[k]
            if st["world"] > 1 or st["force"]:
                dist.all_reduce(self.flat[lo:hi], group=self.group)
        st["done"][k] = True

    def finish(self):
        """Launch the buckets the backward left (parameters without a gradient), join the comm
        stream, scale by 1/world."""
        st = self._armed
        for k in range(len(self.buckets)):
            if not st["done"][k]:
                self._launch(k)
        main = torch.cuda.current_stream(self.flat.device)
        main.wait_stream(st["stream"])
        if st["world"] > 1 or st["force"]:
            self.flat.div_(st["world"])
        self._armed = None
        return self.flat[:self.numel]

    def grads_in_param_order(self) -> torch.Tensor:
        """The gradients (not the guard slot) in ``params`` order."""
        return torch.cat([v.reshape(-1) for v in self.views])


class MetricReducer:
    """The logged per-step scalars, packed and averaged over ranks with one all-reduce."""

    def __init__(self, names: Sequence[str], device, group=None):
        self.names = list(names)
        self.group = group
        self.buf = torch.zeros(len(self.names), dtype=torch.float64, device=device)

    def reduce(self, values: Dict[str, object], world: Optional[int] = None) -> Dict[str, torch.Tensor]:
        for i, k in enumerate(self.names):
            v = values[k]
            self.buf[i] = v.detach().to(self.buf) if torch.is_tensor(v) else float(v)
        world = dist.get_world_size(self.group) if world is None else world
        if world > 1:
            dist.all_reduce(self.buf, group=self.group)
            self.buf.div_(world)
        return {k: self.buf[i] for i, k in enumerate(self.names)}


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None):
    """Rank `src`'s parameters and buffers to every rank (DDP's construction-time broadcast)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)
