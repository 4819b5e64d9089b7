"""The captured training step (fiode_amd.graph_step) replays the same computation as the eager
step: same loss and gradients for the same device Philox counter, fresh draws on every replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


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
