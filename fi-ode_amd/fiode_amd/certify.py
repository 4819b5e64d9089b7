"""Lipschitz certification driver (robustness/certify_lipschitz.py:44-163) on the HIP kernels.

``certify_lipschitz`` keeps the reference loop's semantics per image (init_coordinates -> the
label's decision-boundary grid in ``batches`` slices -> max violation per slice -> certified iff
the max over slices < 0; the "larger T" variant without the grid perturbation), with the grid
built once on the device (``fiode_certify_grid``) and resident in HBM.  Multi-GPU: images are
sharded over ranks (each rank certifies its slice, one all-reduce of the counts at the end);
the per-image computation, including the QP's per-batch global exit, is unchanged by sharding.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import ops
from .streams import new_stream


@dataclass
class CertifyResult:
    n_images: int = 0
    correct: int = 0
    certified: int = 0
    certified_larger_T: int = 0
    max_violations: List[float] = field(default_factory=list)
    certified_idx: List[int] = field(default_factory=list)


def image_shard(n_images: int, rank: int, world: int) -> range:
    """Contiguous image slice of one rank (start_ind/end_ind style)."""
    per = (n_images + world - 1) // world
    lo = min(n_images, rank * per)
    return range(lo, min(n_images, lo + per))


def _record_stream(x, stream) -> None:
    """record_stream on every tensor of a (nested) tuple / list: the caching allocator keeps them
    until `stream` is done with them."""
    if torch.is_tensor(x):
        x.record_stream(stream)
    elif isinstance(x, (tuple, list)):
        for t in x:
            _record_stream(t, stream)


def certify_lipschitz(module, images: torch.Tensor, labels: torch.Tensor, T: int = 40, batches: int = 10,
                      eps: float = 0.141, grid: Optional[torch.Tensor] = None, indices=None) -> CertifyResult:
    """certify_lipschitz.py:97-143 for the given images (module in eval mode, no dropout)."""
    dyn = module.dyn_fun
    dev = images.device
    if grid is None:
        grid = ops.certify_grid(T, device=dev)
    norm = module.init_coordinates.param_map[0]
    min_std = float(norm.std.min()) if getattr(norm, "std", None) is not None else 1.0
    res = CertifyResult()
    module.eval()
    idx = list(range(images.shape[0]) if indices is None else indices)
    labels_h = labels.detach().cpu() if labels.is_cuda else labels       # one host read for all labels
    # The certification kernels of image i run on the current stream while the host is already
    # launching image i + 1's; the validation solve (the accuracy count) runs on a side stream, whose
    # status read (odeint: one host read per solve, as torchdiffeq raises) waits for that stream only,
    # and every result is read once after the loop -- no host round trip between images.
    main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    side = new_stream(dev) if main is not None else None
    pending = []
    with torch.no_grad():
        w = {k: v.detach().float().contiguous() for k, v in dyn.effective_weights().items()}
        cfg = dyn.dyn_cfg()
        cfg.dropout = 0.0
        ts = torch.linspace(0.0, module.t_max, 2, device=dev)
        for i in idx:
            image = images[i:i + 1]
            label = int(labels_h[i])
            # the reference runs module(image) and then init_coordinates(image) again
            # (certify_lipschitz.py:111-113); the backbone is deterministic in eval mode, so its
            # features are computed once and the validation solve starts from them
            static_state, state = module.init_coordinates(image, dyn)
            feats = torch.cuda.Event() if main is not None else None
            if feats is not None:
                feats.record(main)
            out, _ = ops.certify_image(static_state.float().reshape(-1), label, grid, w, cfg, T=T, batches=batches,
                                       eps=eps, min_std=min_std)
            if side is not None:
                side.wait_event(feats)
                _record_stream((static_state, state), side)
                with torch.cuda.stream(side):
                    sol = module.model.integrate_from(static_state, state, ts=ts, int_params=module.val_solver_params)
                    hit = module.model.output_fun(sol)[-1].argmax(-1) == label
                hit.record_stream(main)
            else:
                sol = module.model.integrate_from(static_state, state, ts=ts, int_params=module.val_solver_params)
                hit = module.model.output_fun(sol)[-1].argmax(-1) == label
            pending.append((i, out, hit))
        if main is not None:
            main.wait_stream(side)
        for i, out, hit in pending:
            o = out.cpu()
            vmax, vtmax = float(o[:, 0].max()), float(o[:, 1].max())
            res.n_images += 1
            res.correct += int(hit.item())
            res.max_violations.append(vmax)
            if vmax < 0:
                res.certified += 1
                res.certified_idx.append(int(i))
            if vtmax < 0:
                res.certified_larger_T += 1
    return res


def allreduce_counts(res: CertifyResult, group=None) -> CertifyResult:
    """Sum the per-rank counts with one all-reduce (RCCL on GPU ranks, gloo on CPU)."""
    import torch.distributed as dist
    t = torch.tensor([res.n_images, res.correct, res.certified, res.certified_larger_T], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, group=group)
    t = t.cpu()
    return CertifyResult(int(t[0]), int(t[1]), int(t[2]), int(t[3]), res.max_violations, res.certified_idx)
