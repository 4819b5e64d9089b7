"""The step guard: a poisoned train_ode solve never reaches the parameters (VERDICT r03 Missing #2).

The reference's torchdiffeq loop has no attempt cap and no cross-workgroup exchange, so it never
fails this way; the device solve can (the dopri5 attempt capacity, a timed-out QP-exit exchange),
and then writes NaN into y_hat.  The optimizer kernel reads the solve's status words and the
loss's finiteness on the device and leaves p, m, v and the step counts untouched (torch.amp's
found_inf skip without a host sync); GraphTrainStep.check_status() raises afterwards.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _state(mod, opt):
    ps = [p.detach().clone() for p in mod.parameters()]
    st = [{k: v.detach().clone() for k, v in s.items() if torch.is_tensor(v)} for s in opt.state.values()]
    return ps, st


@pytest.mark.parametrize("kind", ["rk4_exchange_timeout", "dopri5_exchange_timeout", "dopri5_capacity"])
def test_poisoned_solve_leaves_parameters_and_moments(kind, monkeypatch):
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(21)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    if kind == "rk4_exchange_timeout":
        # test hook (common.h): workgroup 1 of the solve never publishes its first exit mask, as if
        # it were not resident; the others time out (~0.5 s), report status 4 and poison y_hat
        monkeypatch.setenv("FIODE_DEBUG_DROP_PUBLISH", "1")
        mod = bench.build_module(dev, seed=0, train_ode=True, solver="rk4")
    elif kind == "dopri5_exchange_timeout":
        # the same hook under the adaptive solve: its float64 batch sums (error ratios) are gathered
        # by every wave for itself, and the poison decision after a timeout must be the same in all
        # waves of a workgroup, or the controller's loop would diverge across the evals'
        # barriers -- the solve has to come back poisoned (status 4), not hang
        monkeypatch.setenv("FIODE_DEBUG_DROP_PUBLISH", "1")
        mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5")
    else:
        mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5")
        mod.train_ode_max_attempts = 1           # the solve needs ~10: capacity exhausted, status 2
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=1)
    assert gs.early                              # the per-layer early updates are guarded too
    before = _state(mod, opt)
    losses = [gs.step().detach().clone() for _ in range(2)]
    torch.cuda.synchronize()
    assert all(not bool(torch.isfinite(lo)) for lo in losses)
    after = _state(mod, opt)
    for a, b in zip(before[0], after[0]):
        assert torch.equal(a, b)
    for sa, sb in zip(before[1], after[1]):
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
    assert gs.skipped_steps() == 2
    assert mod.device_status() == (2 if kind == "dopri5_capacity" else 4)
    with pytest.raises(RuntimeError, match="skipped by the step guard"):
        gs.check_status()


def test_healthy_steps_are_not_skipped():
    """The guard costs nothing on good steps: the guarded replay = an unguarded twin's replay, bit
    for bit (two steps), and no step is counted as skipped."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(22)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    res = []
    for guarded in (True, False):
        mod = bench.build_module(dev, seed=0, train_ode=True)
        mod.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        opt = mod.configure_optimizers(capturable=True)[0][0]
        gs = GraphTrainStep(mod, opt, x, y, warmup=1, guard=guarded)
        assert (opt.guard is not None) == guarded
        losses = [float(gs.step()) for _ in range(2)]
        torch.cuda.synchronize()
        if guarded:
            assert gs.skipped_steps() == 0
            gs.check_status()
        res.append((losses, [p.detach().clone() for p in mod.parameters()]))
        gs.close()
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_adam_kernel_guard_flag():
    """fiode_adam_step with a guard flag: 1 or NaN -> nothing changes (p, m, v, step), the skip
    counted; 0 -> the unguarded update (capturable, device step counts): four guarded steps with
    flags 0, 1, NaN, 0 = two unguarded steps, bit for bit."""
    from fiode_amd.optim import FiodeAdam, StepGuard
    dev = _dev()
    torch.manual_seed(3)
    p0 = [torch.randn(1000, device=dev), torch.randn(17, 5, device=dev)]
    grads = [torch.randn_like(p) for p in p0]
    ps = [torch.nn.Parameter(p.clone()) for p in p0]
    ref = [torch.nn.Parameter(p.clone()) for p in p0]
    opt = FiodeAdam(ps, lr=1e-2, capturable=True)
    topt = FiodeAdam(ref, lr=1e-2, capturable=True)
    flag = torch.zeros(1, device=dev)
    skipped = torch.zeros(1, dtype=torch.int32, device=dev)
    opt.guard = StepGuard(flag=flag, skipped=skipped)
    for it in range(4):
        flag.fill_(1.0 if it == 1 else (float("nan") if it == 2 else 0.0))
        for p, r, gr in zip(ps, ref, grads):
            p.grad = gr.clone()
            r.grad = gr.clone()
        opt.step()
        if it in (0, 3):
            topt.step()
    torch.cuda.synchronize()
    assert int(skipped[0]) == 2
    for p, r in zip(ps, ref):
        assert torch.equal(p, r)
    for p, r in zip(ps, ref):
        sa, sb = opt.state[p], topt.state[r]
        assert float(sa["step"]) == float(sb["step"]) == 2.0
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])


def test_close_disarms_guard_for_eager_steps():
    """After a captured step whose last replay was poisoned (NaN loss, guard verdict 'skip'), close()
    disarms the optimizer's guard: the guard read that replay's graph-pool loss and status words,
    which no eager step writes, so an armed leftover would skip every later step silently.  One
    eager step after close() must move the parameters; a guard=False GraphTrainStep built on the
    same optimizer leaves no guard either."""
    import bench
    from fiode_amd.graph_step import GraphTrainStep
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(23)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    mod = bench.build_module(dev, seed=0, train_ode=True, solver="dopri5")
    mod.train_ode_max_attempts = 1                   # every solve fails: status 2, NaN loss
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=1, check_every=0)
    assert opt.guard is not None
    lo = gs.step()
    torch.cuda.synchronize()
    assert not bool(torch.isfinite(lo)) and gs.skipped_steps() == 1
    gs.close()
    assert opt.guard is None
    mod.train_ode_max_attempts = None                # a healthy eager step
    before = [p.detach().clone() for p in mod.parameters()]
    opt.zero_grad(set_to_none=True)
    loss = mod.compute_loss(x, y, 32, "relu")
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(loss))
    moved = sum(not torch.equal(a, b) for a, b in zip(before, mod.parameters()))
    assert moved >= len(before) // 2, (moved, len(before))        # 0 if a stale guard skipped it
    gs2 = GraphTrainStep(mod, opt, x, y, warmup=1, guard=False)
    assert opt.guard is None
    gs2.close()


def test_guard_refused_with_host_step_counts():
    """A guard on the host-count path (capturable=False) is refused: the host would count a step
    the device then skips, moving the bias correction of every later step."""
    from fiode_amd.optim import FiodeAdam, StepGuard
    dev = _dev()
    p = torch.nn.Parameter(torch.randn(64, device=dev))
    opt = FiodeAdam([p], lr=1e-2, capturable=False)
    opt.guard = StepGuard(flag=torch.zeros(1, device=dev))
    p.grad = torch.randn_like(p)
    with pytest.raises(RuntimeError, match="device step counts"):
        opt.step()
