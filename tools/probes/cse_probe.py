"""Probe (not a test): where the train_ode feature-reuse and the reference-order (backbone run
twice) steps differ."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch
import bench

dev = torch.device("cuda:0")
x = torch.rand(32, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
yb = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(4))
res = {}
for reuse in (True, False, True):
    mod = bench.build_module(dev, seed=0, train_ode=True)
    mod.ode_reuse_features = reuse
    mod._rng_offset = 0
    feats = []
    bb = mod.init_coordinates.param_map
    h = bb.register_forward_hook(lambda m, i, o: feats.append(o.detach().clone()))
    loss = mod.compute_loss(x, yb, 32, "relu")
    h.remove()
    loss.backward()
    torch.cuda.synchronize()
    g = {n: p.grad.detach().clone() for n, p in mod.named_parameters() if p.requires_grad}
    print(reuse, "loss", float(loss), "lyap", float(mod.last_plan["scalars"][0]), "exits",
          mod.last_plan["scalars"][3:5].tolist(), "ode stats", mod.last_ode_plan["stats"].tolist()[:4],
          "n feats", len(feats), flush=True)
    if len(feats) == 2:
        print("  feats equal:", torch.equal(feats[0], feats[1]), float((feats[0] - feats[1]).abs().max()))
    res.setdefault(reuse, []).append((g, feats))
ga = res[True][0][0]; ga2 = res[True][1][0]; gb = res[False][0][0]
for n in ga:
    s = float(ga[n].abs().max()) + 1e-12
    e_rep = float((ga[n] - ga2[n]).abs().max()) / s
    e_cse = float((ga[n] - gb[n]).abs().max()) / s
    if e_rep > 1e-6 or e_cse > 1e-4:
        print(f"{n:60s} repeat {e_rep:.2e}  reuse-vs-ref {e_cse:.2e}")
