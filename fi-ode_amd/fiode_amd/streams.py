"""Dedicated HIP streams for the training step's side branches.

torch.cuda.Stream() hands out streams from a fixed pool (32 per priority, round robin), so a stream
made "fresh" for one role can be the very stream another role already holds: the placement trials
of GraphTrainStep (4 captures, ~9 new side streams each) wrap the pool and alias, e.g., a map-prefetch
stream with the head's weight-gradient stream.  Inside a hipGraph capture that aliasing can make a
stream that joined the capture wait on an event it recorded itself, and this ROCm runtime then
crashes the host in hipStreamEndCapture (a recursive walk of the captured nodes; SIGSEGV under
torch.cuda.graph's capture_end -- tools/probes/capture_selfwait_probe.py reproduces it with four
lines of torch, DESIGN.md "capture_end SIGSEGV").  Every side stream of the product is therefore a
stream of its own, made with hipStreamCreateWithPriority in torch's own HIP runtime and wrapped as
torch.cuda.ExternalStream; they live for the process (a handful per captured step).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HIP = None
_LOCK = threading.Lock()
_MADE: list = []                 # (device index, handle) of every stream made here (never destroyed)


def _hip():
    global _HIP
    if _HIP is None:
        # the runtime instance torch itself uses (a stream of another libamdhip64 would be foreign to it)
        _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        _HIP.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_int]
        _HIP.hipStreamCreateWithPriority.restype = ctypes.c_int
    return _HIP


def new_stream(device, priority: int = 0) -> torch.cuda.Stream:
    """A stream no other role shares (non-blocking, like torch's pool streams; priority as torch's:
    0 normal, -1 high)."""
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    if dev.type != "cuda":
        raise ValueError(f"new_stream: a ROCm device, got {dev}")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    h = ctypes.c_void_p()
    with _LOCK, torch.cuda.device(idx):
        rc = _hip().hipStreamCreateWithPriority(ctypes.byref(h), 1, int(priority))   # 1 = hipStreamNonBlocking
        if rc != 0 or not h.value:
            raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
        _MADE.append((idx, h.value))
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))


def distinct(streams) -> bool:
    """True when no two of ``streams`` (None entries ignored) are the same HIP stream."""
    ids = [s.cuda_stream for s in streams if s is not None]
    return len(ids) == len(set(ids))
