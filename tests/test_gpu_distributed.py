"""Two ranks running the REAL training step (the benched configs[1] step: backbone, Cayley maps,
fused fan-out, train_ode solve, Adam) through GraphTrainStep + GradAllReducer, both on cuda:0 over
gloo -- the DDP semantics of the reference (sl_pipeline.py:157-170; Lightning all-reduces the mean
gradient, and every self.log(..., sync_dist=True) is a mean over ranks, pl_modules.py:451, 483-484):

* after the replayed step each rank's flat gradient bucket equals the mean of the two ranks'
  single-process (eager, same parameters / samples / dropout masks) gradients;
* the fused metric all-reduce gives the per-rank means of the logged scalars;
* each rank's QP exit iterations (batch-global over ITS rows, as under reference DDP) equal its
  solo run's.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "fi-ode_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from fiode_amd.distributed import GradAllReducer, MetricReducer, broadcast_parameters
        from fiode_amd.graph_step import GraphTrainStep
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        B = 32
        mod = bench.build_module(dev, seed=0, train_ode=True)
        mod.seed = 1000 + rank                                  # each rank draws its own samples / masks
        broadcast_parameters(mod)
        g = torch.Generator(device="cpu").manual_seed(77 + rank)
        x = torch.rand(B, 3, 32, 32, generator=g).to(dev)
        y = torch.randint(0, 10, (B,), generator=g).to(dev)
        opt = mod.configure_optimizers(capturable=True)[0][0]
        params = [p for p in mod.parameters() if p.requires_grad]
        reducer = GradAllReducer(params)
        gs = GraphTrainStep(mod, opt, x, y, reducer=reducer, world=world, warmup=2)
        # the solo run: an eager twin with this rank's state right before the replay
        twin = bench.build_module(dev, seed=1, train_ode=True)
        twin.load_state_dict(mod.state_dict())
        twin.rng_counter = mod.rng_counter.clone()
        twin.seed = mod.seed
        for p in twin.parameters():
            p.grad = None
        solo_loss = twin.compute_loss(x, y, B, "relu")
        solo_loss.backward()
        solo = torch.cat([p.grad.reshape(-1) for p in twin.parameters() if p.requires_grad])
        solo_sc = twin.last_plan["scalars"].clone()
        solo_ode = twin.last_ode_plan["stats"].clone()
        gs.step()                                               # replay + RCCL/gloo all-reduce + Adam
        metrics = MetricReducer(["training_loss", "effective_batch_size", "mean_active_constraints"], dev)
        sc = mod.last_plan["scalars"]
        red = metrics.reduce({"training_loss": sc[0], "effective_batch_size": sc[1],
                              "mean_active_constraints": sc[2]}, world)
        torch.cuda.synchronize()
        q.put((rank, dict(bucket=reducer.grads_in_param_order().cpu().numpy().copy(), solo=solo.cpu().numpy(),
                          nbuckets=len(reducer.buckets), comm=gs.comm,
                          solo_sc=solo_sc.cpu().numpy(), sc=sc.cpu().numpy().copy(),
                          solo_ode=solo_ode.cpu().numpy(), ode=mod.last_ode_plan["stats"].cpu().numpy(),
                          red={k: float(v) for k, v in red.items()})))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, RuntimeError(traceback.format_exc())))
    finally:
        dist.destroy_process_group()


def test_two_rank_graph_step_is_ddp_mean():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for v in out.values():
        if isinstance(v, Exception):
            raise v
    a, b = out[0], out[1]
    assert a["comm"] == "eager" and a["nbuckets"] >= 2        # gloo: bucket all-reduces between replays
    assert np.array_equal(a["bucket"], b["bucket"])
    mean = (a["solo"].astype(np.float64) + b["solo"]) / 2
    scale = float(np.abs(mean).max())
    err = float(np.abs(a["bucket"] - mean).max())
    assert err <= 1e-4 * scale, (err, scale)
    for r in (a, b):
        assert (r["sc"][3], r["sc"][4]) == (r["solo_sc"][3], r["solo_sc"][4])     # this rank's QP exits
        assert r["ode"][2] == r["solo_ode"][2]                                    # train_ode last exit
        assert abs(r["sc"][0] - r["solo_sc"][0]) <= 1e-5 * max(1.0, abs(r["solo_sc"][0]))
    for i, k in enumerate(["training_loss", "effective_batch_size", "mean_active_constraints"]):
        exp = (float(a["sc"][i]) + float(b["sc"][i])) / 2
        assert abs(a["red"][k] - exp) <= 1e-6 * max(1.0, abs(exp)) and a["red"][k] == b["red"][k], k


def _world1_main(port, q, comm):
    """One rank on an RCCL ("nccl") group of size 1 with the collectives forced on: the captured
    bucketed all-reduce (comm "graph") must give the same losses and parameters, bit for bit, as
    the single-rank step with the maps refreshed after the optimizer (an all-reduce over one rank
    and the 1/1 scale are exact)."""
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "fi-ode_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    try:
        import bench
        from fiode_amd.distributed import GradAllReducer
        from fiode_amd.graph_step import GraphTrainStep
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        g = torch.Generator(device="cpu").manual_seed(5)
        x = torch.rand(64, 3, 32, 32, generator=g).to(dev)
        y = torch.randint(0, 10, (64,), generator=g).to(dev)
        res = {}
        for mode in ("ref", comm):
            mod = bench.build_module(dev, seed=0, train_ode=True)
            mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
            opt = mod.configure_optimizers(capturable=True)[0][0]
            if mode == "ref":
                gs = GraphTrainStep(mod, opt, x, y, warmup=2)
            elif comm == "graph_placement":
                # the one-graph step with the collectives captured, picked from 3 placements (the
                # decision all-reduced over the ranks; bench.py's N-rank configuration)
                red = GradAllReducer([p for p in mod.parameters() if p.requires_grad])
                gs = GraphTrainStep(mod, opt, x, y, reducer=red, world=1, warmup=2, comm="graph", force_comm=True,
                                    placement_trials=3)
                assert gs.comm == "graph" and len(gs.placement_ms) == 3
            else:
                red = GradAllReducer([p for p in mod.parameters() if p.requires_grad])
                gs = GraphTrainStep(mod, opt, x, y, reducer=red, world=1, warmup=2, comm=comm, force_comm=True)
                assert gs.comm == comm and len(red.buckets) >= 2
            losses = [float(gs.step()) for _ in range(3)]
            torch.cuda.synchronize()
            res[mode] = (losses, [p.detach().cpu().numpy().copy() for p in mod.parameters()])
        q.put((0, dict(ref=res["ref"], got=res[comm])))
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((0, RuntimeError(traceback.format_exc())))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["graph", "eager", "graph_placement"])
def test_world1_rccl_bucketed_allreduce_equals_single(comm):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_main, args=(_free_port(), q, comm))
    p.start()
    import queue
    out = None
    for _ in range(100):                   # a child that dies (e.g. aborted by a runtime error) fails fast
        try:
            _, out = q.get(timeout=1.0)
            break
        except queue.Empty:
            assert p.is_alive() or not q.empty(), f"RCCL child exited with code {p.exitcode}"
    assert out is not None, "RCCL child produced no result in 100 s"
    p.join(timeout=60)
    if isinstance(out, Exception):
        raise out
    (l0, p0), (l1, p1) = out["ref"], out["got"]
    assert l0 == l1
    for a, b in zip(p0, p1):
        assert np.array_equal(a, b)
