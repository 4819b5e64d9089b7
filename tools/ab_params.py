"""A/B bit-identity of whole training steps between two builds of libfiode (not a test):
FIODE_LIB=<lib> python tools/ab_params.py out.pt  runs 4 captured bench steps (train_ode rk4 and
dopri5, B=128, S=256) and saves every parameter and loss; python tools/ab_params.py --cmp a.pt b.pt
compares two outputs."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

if sys.argv[1] == "--cmp":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    bits = lambda t: t.reshape(-1).cpu().view(torch.int32) if t.dtype == torch.float32 else t.reshape(-1).cpu()
    bad = [k for k in a if not torch.equal(bits(a[k]), bits(b[k]))]
    for k in bad[:20]:
        print(k, f"DIFFER max {float((a[k] - b[k]).abs().max())}")
    print(f"{len(a) - len(bad)} of {len(a)} tensors identical")
    sys.exit(1 if bad else 0)

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for solver in ("rk4", "dopri5"):
    mod = bench.build_module(dev, seed=0, train_ode=True, solver=solver)
    mod.seed = 1000
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    gs = GraphTrainStep(mod, opt, x, y)
    for i in range(4):
        out[f"{solver}.loss{i}"] = gs.step().detach().clone()
    torch.cuda.synchronize()
    for n, p in mod.named_parameters():
        out[f"{solver}.{n}"] = p.detach().cpu().clone()
    gs.close()
torch.save(out, sys.argv[1])
print("saved", len(out))
