"""Data-parallel plumbing for the train step and certification (one process per GPU).

The reference trains under Lightning DDP (train_classification.py: ``pl.Trainer(gpus=..,
strategy=DDP)``, ``self.log(..., sync_dist=True)`` in pl_modules.py:480-484): every rank runs the
whole fan-out on its own images, DDP all-reduces the gradients (bucketed, 25 MB) and Lightning
reduces each logged scalar with its own collective.  The path has one real exchange step (the
gradient mean) and one bookkeeping exchange (the logged means), so here:

* ``GradAllReducer``  -- one persistent flat fp32 bucket holding every trainable gradient
  (~2.6 M floats = 10.5 MB for the README model: a single RCCL ring all-reduce, well under one
  xGMI link's latency-bandwidth knee, instead of DDP's per-bucket launches); the views of
  ``p.grad`` point INTO the bucket, so no pack/unpack copies are made.
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
    """Mean of the gradients over ranks with ONE all-reduce of one persistent flat bucket.

    After construction ``p.grad`` of every parameter is a view into ``self.flat`` (the optimizer
    and autograd accumulate into it in place), so ``allreduce()`` is a single collective plus one
    scale, with no gather/scatter copies.  Parameters are laid out in ``parameters()`` order.
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
        self.flat = torch.zeros(self.numel, dtype=self.params[0].dtype, device=dev)
        o = 0
        for p in self.params:
            n = p.numel()
            view = self.flat[o:o + n].view_as(p)
            if p.grad is not None:
                view.copy_(p.grad)
            p.grad = view
            o += n

    def rebind(self):
        """Re-point grads into the bucket (after something replaced p.grad, e.g. set_to_none)."""
        o = 0
        for p in self.params:
            n = p.numel()
            view = self.flat[o:o + n].view_as(p)
            if p.grad is None:
                view.zero_()
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
            p.grad = view
            o += n

    def zero_grad(self):
        self.flat.zero_()

    def gather(self):
        """Move the gradients autograd just produced (fresh tensors: the backward ran with p.grad =
        None, so AccumulateGrad stole its results instead of adding them into the bucket one kernel
        per parameter) into the bucket with ONE multi-tensor copy, and re-point p.grad at the bucket
        views.  A parameter that received no gradient gets zeros."""
        views, o = [], 0
        for p in self.params:
            n = p.numel()
            views.append(self.flat[o:o + n].view_as(p))
            o += n
        have = [(v, p.grad) for v, p in zip(views, self.params) if p.grad is not None]
        if have:
            torch._foreach_copy_([v for v, _ in have], [g for _, g in have])
        for v, p in zip(views, self.params):
            if p.grad is None:
                v.zero_()
            p.grad = v
        return self.flat

    def allreduce(self, world: Optional[int] = None):
        world = dist.get_world_size(self.group) if world is None else world
        if world > 1:
            self.rebind()
            dist.all_reduce(self.flat, group=self.group)
            self.flat.div_(world)
        return self.flat


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
