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


def _bucket_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        import pathlib
        root = pathlib.Path(__file__).resolve().parents[1]
        sys.path[:0] = [str(root), str(root / "fi-ode_amd")]
        from fiode_amd.distributed import GradAllReducer
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.randn(s)) for s in ((300,), (17, 5), (4096,), (3,), (1000, 2))]
        red = GradAllReducer(params)
        g = torch.Generator().manual_seed(10 + rank)
        grads = [torch.randn(p.shape, generator=g) for p in params]
        # the ready order of a backward: reversed parameter order; ~4 KB buckets
        red.plan_buckets(list(reversed(params)), cap_bytes=4096)
        for p, gr in zip(params, grads):
            p.grad.copy_(gr)
        red.allreduce(world)
        q.put((rank, _by_value((len(red.buckets), [p.grad.clone() for p in params], grads,
                                red.grads_in_param_order().clone()))))
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_is_mean_two_ranks():
    """GradAllReducer laid out in a ready order and cut into several buckets: after the bucket
    all-reduces every p.grad (a view into the flat buffer) is the mean of the ranks' gradients."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    nb, g0, raw0, flat0 = out[0]
    _, g1, raw1, _ = out[1]
    g0, g1, raw0, raw1 = ([torch.from_numpy(t) for t in ts] for ts in (g0, g1, raw0, raw1))
    flat0 = torch.from_numpy(flat0)
    assert nb >= 3
    for a, b, r0, r1 in zip(g0, g1, raw0, raw1):
        torch.testing.assert_close(a, (r0 + r1) / 2, rtol=1e-6, atol=1e-7)
        assert torch.equal(a, b)
    assert torch.equal(flat0, torch.cat([g.reshape(-1) for g in g0]))


def _val_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        import pathlib
        root = pathlib.Path(__file__).resolve().parents[1]
        sys.path[:0] = [str(root), str(root / "fi-ode_amd")]
        from fiode_amd.lyapunov import LyapunovLearning

        class _Stub(LyapunovLearning):
            """validation_step's logging with the solve replaced by fixed per-rank outputs (the
            HIP solve needs a GPU; the sync is what is tested)."""
            def __init__(self, out):
                torch.nn.Module.__init__(self)
                self.simplex, self.logged, self._o = True, {}, out

            def forward(self, x, t_steps=2, return_traj=False):
                return self._o

        g = torch.Generator().manual_seed(3 + rank)
        out = torch.softmax(torch.randn(16, 10, generator=g), -1)
        y = torch.randint(0, 10, (16,), generator=g)
        m = _Stub(out)
        m.validation_step((torch.zeros(16, 3, 32, 32), y))
        local_loss = torch.nn.functional.nll_loss(torch.log(out), y)
        local_err = (out.argmax(-1) != y).float().mean()
        q.put((rank, ({k: float(v) for k, v in m.logged.items()}, float(local_loss), float(local_err))))
    finally:
        dist.destroy_process_group()


def test_validation_metrics_synced_two_ranks():
    """validation_step logs validation_loss / error / adv_error with sync_dist=True
    (pl_modules.py:217-219): every rank logs the mean over ranks."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_val_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    (l0, a0, e0), (l1, a1, e1) = out[0], out[1]
    assert l0 == l1
    assert abs(l0["validation_loss"] - (a0 + a1) / 2) < 1e-6
    assert abs(l0["validation_error"] - (e0 + e1) / 2) < 1e-6
    assert l0["validation_adv_error"] == l0["validation_error"]


def test_graph_step_refuses_too_few_hw_queues(monkeypatch):
    """GPU_MAX_HW_QUEUES < 4: the HIP runtime's graph executor segfaults replaying a multi-branch graph
    (tools/probes/hwq_branch_probe.py), so GraphTrainStep refuses before capturing anything."""
    import torch
    from fiode_amd.graph_step import GraphTrainStep
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    with pytest.raises(RuntimeError, match="GPU_MAX_HW_QUEUES=2"):
        GraphTrainStep(None, None, torch.zeros(1), torch.zeros(1))
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    with pytest.raises(ValueError, match="ROCm device"):       # passes the queue check, then needs a GPU
        GraphTrainStep(None, None, torch.zeros(1), torch.zeros(1))
