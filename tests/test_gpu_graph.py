"""The captured training step (fiode_amd.graph_step) replays the same computation as the eager
step: same loss and gradients for the same device Philox counter, fresh draws on every replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _copy_inv_cache(src, dst):
    """The dense Cayley maps' warm-start inverses (cayley._warm_inverse) are step state too: the twin
    that replays a step eagerly starts from the same ones."""
    from fiode_amd.cayley import CayleyLinear
    for a, b in zip([m for m in src.modules() if isinstance(m, CayleyLinear)],
                    [m for m in dst.modules() if isinstance(m, CayleyLinear)]):
        b._inv_cache = {k: v.detach().clone() for k, v in a._inv_cache.items() if torch.is_tensor(v)}


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
    gs = GraphTrainStep(mod, opt, x, y, warmup=2)
    twin = bench.build_module(dev, seed=1, train_ode=train_ode)          # same parameters / counter as before the replay
    twin.load_state_dict(mod.state_dict())
    twin.rng_counter = mod.rng_counter.clone()
    twin.seed = mod.seed
    _copy_inv_cache(mod, twin)
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
    _copy_inv_cache(mod, twin)
    topt = twin.configure_optimizers(capturable=True)[0][0]
    gs.step()
    topt.zero_grad(set_to_none=True)
    twin.compute_loss(x, y, 32, "relu").backward()
    topt.step()
    torch.cuda.synchronize()
    for (k, a), b in zip(mod.named_parameters(), twin.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=k)


@pytest.mark.parametrize("train_ode", [False, True])
def test_maps_ahead_equal_step_start_maps(train_ode):
    """GraphTrainStep(maps_ahead=True) -- each conv layer's Cayley map for the next step computed
    inside the current one, right after the layer's early Adam update -- gives the same losses and
    parameters, bit for bit, as maps computed at the start of every step, over several replays."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    out = {}
    for ahead in ("conv", "conv+linear", "conv+small", None):
        mod = bench.build_module(dev, seed=0, train_ode=train_ode)
        mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        opt = mod.configure_optimizers(capturable=True)[0][0]
        gs = GraphTrainStep(mod, opt, x, y, warmup=2, maps_ahead=ahead is not None,
                            maps_ahead_linear={"conv+linear": True, "conv+small": "small"}.get(ahead, False))
        assert len(gs.piped) == {"conv": 4, "conv+linear": 7, "conv+small": 5, None: 0}[ahead]
        losses = [float(gs.step()) for _ in range(3)]
        torch.cuda.synchronize()
        out[ahead] = (losses, [p.detach().clone() for p in mod.parameters()])
        gs.close()
    for ahead in ("conv", "conv+linear", "conv+small"):
        assert out[ahead][0] == out[None][0], ahead
        for a, b in zip(out[ahead][1], out[None][1]):
            assert torch.equal(a, b), ahead
