"""FiodeAdam / FiodeAdamW (adam.hip, one launch over all parameter tensors) against torch.optim.Adam
/ AdamW on the same gradients: the update formula is torch's fused Adam in the same operation
order, so results agree to fp32 rounding (torch's kernel may contract multiply-adds: tolerance
below).  Covers sizes that are not multiples of 4, a misaligned view (scalar path), weight decay
(coupled and decoupled), maximize, device (capturable) and host step counts, and a hipGraph
capture of the step replayed against eager steps."""
import pytest
import torch

from fiode_amd.optim import FiodeAdam, FiodeAdamW

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
RTOL, ATOL = 1e-5, 1e-7


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    flat = torch.randn(4096 + 1, generator=g)
    shapes = [(512, 512), (10,), (1,), (3, 5), (1025,), (128, 10)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ps.append(flat[1:1 + 999].clone().view(999))          # odd length
    base = flat.to(DEV)
    return ps, base


def _run(kind, steps, **kw):
    ps, base = _params(0)
    a = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    b = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    # a misaligned view (offset 1 float): the kernel's scalar path
    mis_a = torch.nn.Parameter(base[1:1 + 777].clone())
    a.append(mis_a)
    b.append(torch.nn.Parameter(mis_a.detach().clone()))
    ours = (FiodeAdamW if kind == "adamw" else FiodeAdam)(a, **kw)
    ref = (torch.optim.AdamW if kind == "adamw" else torch.optim.Adam)(b, **kw)
    g = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(steps):
        for x, y in zip(a, b):
            gr = torch.randn(x.shape, generator=g, device=DEV)
            x.grad, y.grad = gr.clone(), gr.clone()
        ours.step()
        ref.step()
    torch.cuda.synchronize()
    return a, b, ours, ref


@pytest.mark.parametrize("kind,kw", [
    ("adam", dict(lr=5e-3)),
    ("adam", dict(lr=1e-3, weight_decay=5e-4, betas=(0.8, 0.99))),
    ("adam", dict(lr=1e-3, maximize=True, capturable=True)),
    ("adam", dict(lr=1e-3, fused=True, capturable=True)),
    ("adamw", dict(lr=2e-3, weight_decay=1e-2)),
    ("adamw", dict(lr=2e-3, weight_decay=1e-2, fused=True, capturable=True)),
])
def test_fiode_adam_matches_torch(kind, kw):
    a, b, ours, ref = _run(kind, 5, **kw)
    for x, y in zip(a, b):
        torch.testing.assert_close(x.detach(), y.detach(), rtol=RTOL, atol=ATOL)
    for sx, sy in zip(ours.state.values(), ref.state.values()):
        torch.testing.assert_close(sx["exp_avg"], sy["exp_avg"], rtol=RTOL, atol=ATOL)
        torch.testing.assert_close(sx["exp_avg_sq"], sy["exp_avg_sq"], rtol=RTOL, atol=1e-12)
        assert float(sx["step"]) == float(sy["step"]) == 5.0


def test_fiode_adam_graph_replay_equals_eager():
    ps, _ = _params(3)
    a = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    b = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    oa = FiodeAdam(a, lr=1e-3, capturable=True)
    ob = FiodeAdam(b, lr=1e-3, capturable=True)
    grads = [torch.zeros_like(x) for x in a]
    for x, gr in zip(a, grads):
        x.grad = gr
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        oa.step()                                  # warm-up: creates the state outside the capture
    torch.cuda.current_stream().wait_stream(s)
    ob_grads = [torch.zeros_like(x) for x in b]
    for y, gr in zip(b, ob_grads):
        y.grad = gr
    ob.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        oa.step()
    g = torch.Generator(device=DEV).manual_seed(5)
    for _ in range(4):
        for gr, gb in zip(grads, ob_grads):
            r = torch.randn(gr.shape, generator=g, device=DEV)
            gr.copy_(r)
            gb.copy_(r)
        graph.replay()
        ob.step()
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x.detach(), y.detach())
    assert float(oa.state[a[0]]["step"]) == 5.0


def test_tensor_lr_followed_by_captured_step():
    """A tensor lr (torch's capturable LR scheduling: schedulers update it in place) is read by the
    kernel on the device, so a captured step follows a change made between replays; the values equal
    torch's Adam run eagerly with the same float lr sequence."""
    ps, _ = _params(4)
    a = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    b = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    lr_t = torch.tensor(1e-3, device=DEV)
    oa = FiodeAdam(a, lr=lr_t, capturable=True)
    ob = torch.optim.Adam(b, lr=1e-3, capturable=True)
    grads = [torch.zeros_like(x) for x in a]
    for x, gr in zip(a, grads):
        x.grad = gr
    for y in b:
        y.grad = torch.zeros_like(y)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        oa.step()
    torch.cuda.current_stream().wait_stream(s)
    ob.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        oa.step()
    g = torch.Generator(device=DEV).manual_seed(6)
    for lr in (1e-3, 4e-3, 2.5e-4):
        lr_t.fill_(lr)                              # what CosineAnnealingLR / MultiStepLR do to a tensor lr
        for pg in ob.param_groups:
            pg["lr"] = lr
        for gr, y in zip(grads, b):
            r = torch.randn(gr.shape, generator=g, device=DEV)
            gr.copy_(r)
            y.grad.copy_(r)
        graph.replay()
        ob.step()
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        torch.testing.assert_close(x.detach(), y.detach(), rtol=RTOL, atol=ATOL)
