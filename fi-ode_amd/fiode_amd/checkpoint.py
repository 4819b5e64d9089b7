"""Checkpoint compatibility with the reference's Lightning `.ckpt` files.

The reference restores trained modules with
``ModuleType.load_from_checkpoint(chkpt_file, map_location=..., strict=False, **cfg)``
(robustness/eval_utils.py:92-107, utils.py:14-28): Lightning builds the module from the hydra config
and loads ``ckpt["state_dict"]`` into it.  The module tree here keeps the reference's names, so the
same keys land in the same places:

* ``model.dyn_fun.{hidden_to_mlp,mlp_to_mlp,mlp_to_hidden,U_x}.{weight,bias,alpha}``
  (classification.py:44-83; CayleyLinear's ``alpha``), ``singular_u`` buffers when present
  (LipsLinear, classification.py:19-28) -- a None buffer is absent from a state_dict on both sides;
* ``model.init_coordinates.h0_0`` (init_coordinates.py:38-44) and
  ``model.init_coordinates.param_map.*`` (the backbone; its inner names follow the restated
  KWLarge_Concat, because libs/ortho_conv is absent: parity of the backbone keys is unpinned);
* ``model.ts`` (models.py:195-199).

Files are read with ``torch.load(weights_only=True)`` only -- a checkpoint that needs unpickling of
arbitrary objects is refused, never executed.  Cayley maps are recomputed from the parameters on
every training forward; a map already prefetched on a side stream (``_pre``) is dropped by a load,
and a loaded CayleyConv ``alpha`` is kept (no data-dependent re-initialisation).

``save_checkpoint`` writes the same layout (``state_dict`` + ``epoch`` / ``global_step`` +
optimizer states), so a run can be checkpointed here and resumed here or loaded by the reference.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Iterable, Optional, Tuple

import torch
from torch import nn

LIGHTNING_VERSION = "1.6.0"   # the version string the reference environment records (env.yml)


class CheckpointError(RuntimeError):
    pass


def read_checkpoint(path: str | os.PathLike, map_location: Any = "cpu") -> Dict[str, Any]:
    """The checkpoint dict, read without executing anything from the file."""
    try:
        ck = torch.load(path, map_location=map_location, weights_only=True)
    except Exception as e:  # weights_only refusal or a corrupt file: say which file and why
        raise CheckpointError(f"cannot read {path} with torch.load(weights_only=True): {e}") from e
    if not isinstance(ck, dict):
        raise CheckpointError(f"{path}: expected a dict checkpoint, got {type(ck).__name__}")
    return ck


def checkpoint_state_dict(ck: Dict[str, Any]) -> Dict[str, torch.Tensor]:
    """``ckpt["state_dict"]`` for a Lightning file, the dict itself for a bare state_dict."""
    sd = ck.get("state_dict", ck)
    bad = [k for k, v in sd.items() if not isinstance(v, torch.Tensor)]
    if bad:
        raise CheckpointError(f"non-tensor entries in the state_dict: {bad[:5]}")
    return sd


def load_state(module: nn.Module, state_dict: Dict[str, torch.Tensor], strict: bool = False
               ) -> Tuple[list, list]:
    """``module.load_state_dict`` with Lightning's strict semantics, shape mismatches always raised
    (Lightning's strict=False only tolerates missing / unexpected keys).  Returns
    (missing_keys, unexpected_keys)."""
    own = module.state_dict()
    shape_bad = [(k, tuple(v.shape), tuple(own[k].shape)) for k, v in state_dict.items()
                 if k in own and tuple(own[k].shape) != tuple(v.shape)]
    if shape_bad:
        raise CheckpointError("shape mismatch (key, checkpoint, module): " + "; ".join(map(str, shape_bad[:5])))
    res = module.load_state_dict(state_dict, strict=strict)
    for m in module.modules():          # Cayley maps prefetched from the old weights are stale
        if getattr(m, "_pre", None) is not None:
            m._pre = None
    return list(res.missing_keys), list(res.unexpected_keys)


def load_from_checkpoint(module: nn.Module, path: str | os.PathLike, strict: bool = False,
                         map_location: Any = None) -> Dict[str, Any]:
    """Load a reference (or our own) checkpoint into an already-built module (the module side of
    ``hydra_conf_load_from_checkpoint_nonstrict``).  Tensors are moved to the module's device.
    Returns {"missing_keys", "unexpected_keys", "epoch", "global_step"}."""
    ck = read_checkpoint(path, map_location="cpu" if map_location is None else map_location)
    sd = checkpoint_state_dict(ck)
    missing, unexpected = load_state(module, sd, strict=strict)
    return dict(missing_keys=missing, unexpected_keys=unexpected, epoch=ck.get("epoch"),
                global_step=ck.get("global_step"))


def save_checkpoint(module: nn.Module, path: str | os.PathLike, epoch: int = 0, global_step: int = 0,
                    optimizers: Optional[Iterable[torch.optim.Optimizer]] = None,
                    extra: Optional[Dict[str, Any]] = None) -> None:
    """Lightning-layout checkpoint: only tensors and plain containers, so it reads back with
    weights_only=True here and with Lightning's loader in the reference."""
    sd = {k: v.detach().cpu() for k, v in module.state_dict().items()}
    ck: Dict[str, Any] = {"epoch": int(epoch), "global_step": int(global_step),
                          "pytorch-lightning_version": LIGHTNING_VERSION, "state_dict": sd}
    if optimizers is not None:
        ck["optimizer_states"] = [_cpu(o.state_dict()) for o in optimizers]
    if extra:
        ck.update(extra)
    tmp = f"{path}.tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)           # a crash mid-write never leaves a truncated checkpoint


def restore_training_state(module: nn.Module, path: str | os.PathLike,
                           optimizers: Optional[Iterable[torch.optim.Optimizer]] = None) -> Dict[str, Any]:
    """Resume: weights (strict), optimizer states, and the epoch / global_step counters the loss
    reads (kappa ramp, sampler mixing, scale_nominal switch)."""
    info = load_from_checkpoint(module, path, strict=True)
    ck = read_checkpoint(path)
    if optimizers is not None:
        states = ck.get("optimizer_states")
        optimizers = list(optimizers)
        if states is None or len(states) != len(optimizers):
            raise CheckpointError(f"{path}: {0 if states is None else len(states)} optimizer states for "
                                  f"{len(optimizers)} optimizers")
        for o, s in zip(optimizers, states):
            o.load_state_dict(s)
    if hasattr(module, "current_epoch") and info["epoch"] is not None:
        module.current_epoch = int(info["epoch"])
    if hasattr(module, "global_step") and info["global_step"] is not None:
        module.global_step = int(info["global_step"])
    return info


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj
