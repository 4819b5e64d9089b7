"""ops._Workspace (host logic, CPU tensors): cached per (device, tag), never freed once replaced (a
captured graph may replay into it), and zeroed buffers first asked for inside a capture taken from
the arena reserved -- and zeroed -- before it, never from the capture's own pool."""
import sys
from pathlib import Path

import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fi-ode_amd"))


@pytest.fixture()
def ws(monkeypatch):
    from fiode_amd import ops
    W = ops._Workspace
    monkeypatch.setattr(W, "_cache", {})
    monkeypatch.setattr(W, "_arena", {})
    monkeypatch.setattr(W, "_zero_max", {})
    monkeypatch.setattr(W, "_retired", [])
    monkeypatch.setattr(W, "fills_in_capture", 0)
    capturing = {"on": False}
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: capturing["on"])
    return W, capturing


def test_cached_grown_and_retired(ws):
    W, _ = ws
    dev = torch.device("cpu")
    a = W.get(dev, 1000, "t", zero=True)
    assert a.numel() >= 1000 and int(a.sum()) == 0
    assert W.get(dev, 500, "t", zero=True) is a            # large enough: the same buffer
    b = W.get(dev, 4000, "t", zero=True)
    assert b is not a and b.numel() >= 4000
    assert any(r is a for r in W._retired)                 # kept alive, never freed
    assert W.get(dev, 100, "other").numel() >= 256         # minimum size, own tag


def test_capture_takes_reserved_zeroed_slots(ws):
    W, capturing = ws
    dev = torch.device("cpu")
    W.get(dev, 3000, "warmup", zero=True)                  # the eager warm-up's largest zeroed request
    W.reserve(dev, slots=2)
    arena = W._arena[None][0]
    arena[:] = 0
    capturing["on"] = True
    s1 = W.get(dev, 2000, "stream1", zero=True)
    s2 = W.get(dev, 3000, "stream2", zero=True)
    assert s1.data_ptr() == arena.data_ptr()               # slot 0 of the arena
    assert s2.data_ptr() == arena.data_ptr() + W._arena[None][1]
    assert W.fills_in_capture == 0
    s3 = W.get(dev, 1000, "stream3", zero=True)            # arena exhausted: the capture fills
    assert W.fills_in_capture == 1 and int(s3.sum()) == 0
    s4 = W.get(dev, 10000, "stream4", zero=True)           # larger than a slot: fills too
    assert W.fills_in_capture == 2 and s4.numel() >= 10000
    capturing["on"] = False
    assert W.get(dev, 2000, "stream1", zero=True) is s1    # the stream keeps its slot
