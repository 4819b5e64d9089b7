"""world_size-2 gloo tests of the data-parallel plumbing (fiode_amd/distributed.py, certify shards)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _by_value(obj):
    """Tensors cross the queue as numpy copies: a shared-memory tensor handle would need the
    worker alive until the parent unpickles it (EOFError when the worker exits first)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy().copy()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_by_value(o) for o in obj)
    return obj


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _by_value(fn(rank, world))))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in out.items():
        if isinstance(v, Exception):
            raise v
    return out


def _grad_case(rank, world):
    import sys, pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "fi-ode_amd"))
    from fiode_amd.distributed import GradAllReducer, broadcast_parameters
    torch.manual_seed(rank)                                   # different init per rank ...
    m = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    broadcast_parameters(m)                                   # ... made equal by the broadcast
    red = GradAllReducer(m.parameters())
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(4, 7, generator=g)
    m(x).pow(2).sum().backward()
    local = [p.grad.clone() for p in m.parameters()]
    red.allreduce()
    return [p.detach().clone() for p in m.parameters()], local, [p.grad.clone() for p in m.parameters()], \
        red.flat.data_ptr() == m[0].weight.grad.data_ptr()


def test_grad_allreduce_mean_two_ranks():
    out = _run(_grad_case)
    (p0, l0, g0, alias0), (p1, l1, g1, alias1) = out[0], out[1]
    assert alias0 and alias1
    T = torch.from_numpy
    for a, b in zip(p0, p1):
        assert torch.equal(T(a), T(b))
    for a, b, la, lb in zip(g0, g1, l0, l1):
        assert torch.equal(T(a), T(b))
        torch.testing.assert_close(T(a), (T(la) + T(lb)) / 2)


def _metric_case(rank, world):
    import sys, pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "fi-ode_amd"))
    from fiode_amd.distributed import MetricReducer
    r = MetricReducer(["loss", "ebs", "mac"], device="cpu")
    out = r.reduce({"loss": torch.tensor(1.0 + rank), "ebs": 10.0 * rank, "mac": 3.0})
    return {k: float(v) for k, v in out.items()}


def test_metric_reduce_two_ranks():
    out = _run(_metric_case)
    assert out[0] == out[1] == {"loss": 1.5, "ebs": 5.0, "mac": 3.0}


def _cert_case(rank, world):
    import sys, pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "fi-ode_amd"))
    from fiode_amd.certify import CertifyResult, allreduce_counts, image_shard
    sh = image_shard(7, rank, world)
    res = CertifyResult(n_images=len(sh), correct=len(sh) - rank, certified=rank + 1, certified_larger_T=1)
    tot = allreduce_counts(res)
    return list(sh), (tot.n_images, tot.correct, tot.certified, tot.certified_larger_T)


def test_certify_counts_two_ranks():
    out = _run(_cert_case)
    assert out[0][0] + out[1][0] == list(range(7))
    assert out[0][1] == out[1][1] == (7, 6, 3, 2)


def test_shard_range_covers_exactly():
    from fiode_amd.distributed import shard_range
    for n in (0, 1, 5, 8, 127, 10000):
        for w in (1, 2, 3, 8):
            seen = [i for r in range(w) for i in shard_range(n, r, w)]
            assert seen == list(range(n))
