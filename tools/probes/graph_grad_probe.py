import sys, pathlib
ROOT = pathlib.Path("/root/repo")
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch, bench
from fiode_amd.graph_step import GraphTrainStep
dev = torch.device("cuda:0")
for train_ode in (True,):
    mod = bench.build_module(dev, seed=0, train_ode=train_ode)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.rand(32, 3, 32, 32, generator=g).to(dev); y = torch.randint(0, 10, (32,), generator=g).to(dev)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    gs = GraphTrainStep(mod, opt, x, y, warmup=2)
    twin = bench.build_module(dev, seed=1, train_ode=train_ode)
    twin.load_state_dict(mod.state_dict()); twin.rng_counter = mod.rng_counter.clone(); twin.seed = mod.seed
    loss = gs.step(); torch.cuda.synchronize()
    gg = {n: p.grad.clone() for n, p in mod.named_parameters() if p.requires_grad}
    for p in twin.parameters(): p.grad = None
    l2 = twin.compute_loss(x, y, 32, "relu"); l2.backward()
    print("loss", float(loss), float(l2))
    for n, p in twin.named_parameters():
        if not p.requires_grad: continue
        a, b = gg[n], p.grad
        d = float((a - b).abs().max()); r = float(b.abs().max())
        if d > 1e-5 + 1e-4 * r: print("MISMATCH", n, d, r)
print("done")
