"""The captured training step (fiode_amd.graph_step) replays the same computation as the eager
step: same loss and gradients for the same device Philox counter, fresh draws on every replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


@pytest.mark.filterwarnings("error:.*AccumulateGrad node's stream.*:UserWarning")
@pytest.mark.parametrize("train_ode", [False, True])
def test_graph_replay_matches_eager_step(train_ode):
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    mod = bench.build_module(dev, seed=0, train_ode=train_ode)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    # one capture, so that the AccumulateGrad-stream check above holds (the default warm capture
    # binds the parameters' accumulators to its own stream on purpose: graph_step.py)
    gs = GraphTrainStep(mod, opt, x, y, warmup=2, warm_capture=False)
    twin = bench.build_module(dev, seed=1, train_ode=train_ode)          # same parameters / counter as before the replay
    twin.load_state_dict(mod.state_dict())
    twin.rng_counter = mod.rng_counter.clone()
    twin.seed = mod.seed
    c0 = int(mod.rng_counter)
    loss = gs.step()
    torch.cuda.synchronize()
    assert int(mod.rng_counter) == c0 + 1
    graph_grads = [p.grad.clone() for p in mod.parameters() if p.requires_grad]
    for p in twin.parameters():
        p.grad = None
    l2 = twin.compute_loss(x, y, 32, "relu")
    l2.backward()
    eager_grads = [p.grad for p in twin.parameters() if p.requires_grad]
    torch.testing.assert_close(loss, l2, rtol=1e-5, atol=1e-6)
    for a, b in zip(graph_grads, eager_grads):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    # fresh samples on the next replay
    before = float(loss)
    after = float(gs.step())
    assert after != before


def test_graph_warmup_leaves_no_updates():
    """Constructing GraphTrainStep (warm-up iterations + capture) leaves the parameters, the Adam
    state and the Philox counter as they were; the first replay then equals one eager training
    step (compute_loss + backward + Adam) from the same state."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    mod = bench.build_module(dev, seed=0, train_ode=False)
    g = torch.Generator(device="cpu").manual_seed(6)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    before = {k: v.detach().clone() for k, v in mod.state_dict().items()}
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=3)
    torch.cuda.synchronize()
    for k, v in mod.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert int(mod.rng_counter) == 0
    for st in opt.state.values():
        for k, v in st.items():
            if torch.is_tensor(v):
                assert int(torch.count_nonzero(v)) == 0, k
    # one replay == one eager step from the same state
    twin = bench.build_module(dev, seed=1, train_ode=False)
    twin.load_state_dict(before)
    twin.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    twin.seed = mod.seed
    topt = twin.configure_optimizers(capturable=True)[0][0]
    gs.step()
    topt.zero_grad(set_to_none=True)
    twin.compute_loss(x, y, 32, "relu").backward()
    topt.step()
    torch.cuda.synchronize()
    for (k, a), b in zip(mod.named_parameters(), twin.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=k)


@pytest.mark.parametrize("train_ode,reuse", [(False, True), (True, True), (True, False)])
def test_maps_ahead_equal_step_start_maps(train_ode, reuse):
    """GraphTrainStep(maps_ahead=True) -- each conv layer's Cayley map for the next step computed
    inside the current one, right after the layer's early Adam update -- gives the same losses and
    parameters, bit for bit, as maps computed at the start of every step, over several replays.
    With the reference-order second backbone pass (ode_reuse_features False) every conv map is used
    twice per step: there the early per-layer update is off and the maps are refreshed after the
    optimizer step (still bit-identical)."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    out = {}
    for ahead in (True, False):
        mod = bench.build_module(dev, seed=0, train_ode=train_ode)
        mod.ode_reuse_features = reuse
        mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        opt = mod.configure_optimizers(capturable=True)[0][0]
        gs = GraphTrainStep(mod, opt, x, y, warmup=2, maps_ahead=ahead)
        assert len(gs.piped) == (4 if ahead else 0)
        assert gs.early == (ahead and (reuse or not train_ode))
        losses = [float(gs.step()) for _ in range(3)]
        torch.cuda.synchronize()
        out[ahead] = (losses, [p.detach().clone() for p in mod.parameters()])
        gs.close()
    assert out[True][0] == out[False][0]
    for a, b in zip(out[True][1], out[False][1]):
        assert torch.equal(a, b)


def test_float_lr_change_refused_tensor_lr_followed():
    """A float lr is baked into the captured optimizer step: changing it after capture makes step()
    raise instead of silently replaying the old value.  A tensor lr (capturable LR scheduling) is read
    on the device: a scheduler's in-place change is followed by the replays (the replayed step equals
    an eager step of a twin at the new lr)."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(8)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    mod = bench.build_module(dev, seed=0, train_ode=False)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=1)
    gs.step()
    opt.param_groups[0]["lr"] = 1e-3
    with pytest.raises(RuntimeError, match="learning rate changed"):
        gs.step()
    gs.close()
    from fiode_amd.optim import FiodeAdam
    res = {}
    for lr_kind in ("tensor", "float"):
        m = bench.build_module(dev, seed=0, train_ode=False)
        m.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        params = list(m.parameters())
        lr0 = torch.tensor(5e-3, device=dev) if lr_kind == "tensor" else 5e-3
        o = FiodeAdam(params, lr=lr0, capturable=True, fused=True)
        if lr_kind == "tensor":
            st = GraphTrainStep(m, o, x, y, warmup=1)
            st.step()
            lr0.fill_(1e-3)                      # what a scheduler does to a tensor lr
            st.step()
            st.close()
        else:
            st = GraphTrainStep(m, o, x, y, warmup=1)
            st.step()
            st.close()
            for pg in o.param_groups:
                pg["lr"] = 1e-3
            st = GraphTrainStep(m, o, x, y, warmup=1)      # recapture at the new float lr
            st.step()
            st.close()
        torch.cuda.synchronize()
        res[lr_kind] = [p.detach().clone() for p in params]
    for a, b in zip(res["tensor"], res["float"]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_graph_replays_without_runtime_queue_override():
    """The captured configs[1] step (bench shape: B=128, S=256, train_ode rk4) replays correctly
    with the HIP runtime's own graph-executor settings: DEBUG_HIP_FORCE_GRAPH_QUEUES is not set in
    this process (bench.py sets it only as a tuning default when run as the program).  30 replays,
    every loss finite, the device status clean."""
    import os
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    assert "DEBUG_HIP_FORCE_GRAPH_QUEUES" not in os.environ
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    mod = bench.build_module(dev, seed=0, train_ode=True)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y)
    losses = torch.stack([gs.step().detach().clone() for _ in range(30)])
    torch.cuda.synchronize()
    assert bool(torch.isfinite(losses).all())
    gs.check_status()
    assert mod.device_status() == 0


def test_kappa_ramp_followed_by_captured_step():
    """kappa_length > 0 (pl_modules.py:447-448: kappa = global_step / kappa_length * kappa while
    global_step < kappa_length): the captured step reads kappa from the device step counter, so its
    replays follow the ramp -- equal to eager steps of a twin at the host's kappa (losses 1e-5,
    parameters 1e-4 after 3 steps); the ramp is visible in the loss (kappa 0, 0.2, 0.4)."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(12)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    mods = []
    for seed in (0, 1):
        m = bench.build_module(dev, seed=seed, train_ode=False)
        m.dyn_fun.kappa_length = 10
        m.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        mods.append(m)
    mod, twin = mods
    twin.load_state_dict(mod.state_dict())
    twin.seed = mod.seed
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=2)
    topt = twin.configure_optimizers(capturable=True)[0][0]
    for step in range(3):
        assert twin.current_kappa() == step / 10 * 2.0
        loss = float(gs.step())
        topt.zero_grad(set_to_none=True)
        l2 = twin.compute_loss(x, y, 32, "relu")
        l2.backward()
        topt.step()
        twin.global_step += 1
        twin.rng_counter.add_(1)
        torch.cuda.synchronize()
        assert abs(loss - float(l2)) <= 1e-5 * max(1.0, abs(loss)), (step, loss, float(l2))
    assert mod.global_step == 3
    for a, b in zip(mod.parameters(), twin.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    gs.close()


def test_placement_trials_keep_results_bit_identical():
    """GraphTrainStep(placement_trials=3) -- captures on fresh side streams, the fastest kept, the
    trial replays' updates undone -- replays the same losses and parameters, bit for bit, as a
    single capture from the same state."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    out = {}
    for trials in (1, 3):
        mod = bench.build_module(dev, seed=0, train_ode=True)
        mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        opt = mod.configure_optimizers(capturable=True)[0][0]
        gs = GraphTrainStep(mod, opt, x, y, warmup=2, placement_trials=trials)
        assert (gs.placement_ms is None) == (trials == 1)
        assert int(mod.rng_counter) == 0 and mod.global_step == 0
        losses = [float(gs.step()) for _ in range(3)]
        torch.cuda.synchronize()
        out[trials] = (losses, [p.detach().clone() for p in mod.parameters()])
        gs.close()
    assert len(out[3][0]) == 3 and out[1][0] == out[3][0]
    for a, b in zip(out[1][1], out[3][1]):
        assert torch.equal(a, b)


def test_placement_trials_use_distinct_dedicated_streams():
    """The placement trials' fresh side streams are streams of their own (fiode_amd.streams), never
    torch pool streams that could alias another role's stream: after the trials every role stream of
    the kept capture is a distinct HIP stream, and the capture-time check refuses an aliased one."""
    import bench
    from fiode_amd import cayley as CY, streams
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    mod = bench.build_module(dev, seed=0, train_ode=True)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    from fiode_amd import ops
    fills = ops._Workspace.fills_in_capture
    gs = GraphTrainStep(mod, opt, x, y, warmup=2, placement_trials=4)
    roles = [s for s in gs.role_streams() if s is not None]
    assert len(roles) >= 8 and streams.distinct(roles)
    # every zeroed GEMM workspace of the 5 captures came from a reserved arena (no captured fill)
    assert ops._Workspace.fills_in_capture == fills
    gs.step()
    torch.cuda.synchronize()
    mod._wtap_stream = CY._head_stream(dev)          # two roles on one stream: refused before capturing
    with pytest.raises(RuntimeError, match="share one HIP stream"):
        gs._capture()
    gs.close()
