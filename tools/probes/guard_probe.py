"""Which replayed step does the step guard skip, and why (not a test): the bench's configs[2]
module (train_ode dopri5), GraphTrainStep, per step the loss, the solve's
stats (nfe, status, accepted / rejected, attempts), its status word and the skip count."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402


def run(solver: str, steps: int = 30, B: int = 128, S: int = bench.H_SAMPLE):
    dev = torch.device("cuda:0")
    mod = bench.build_module(dev, seed=0, train_ode=True, solver=solver, h_sample=S)
    mod.seed = 1000
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(B, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (B,), generator=g).to(dev)
    gs = GraphTrainStep(mod, opt, x, y, check_every=0)
    print(f"== solver={solver}", flush=True)
    prev = 0
    for i in range(steps):
        t0 = time.perf_counter()
        loss = gs.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        st = mod.last_ode_plan["stats"].cpu().tolist()
        sw = mod.last_ode_plan.get("status_word")
        sk = gs.skipped_steps()
        flag = " <-- skipped" if sk != prev else ""
        prev = sk
        pl = mod.last_plan
        yh = pl.get("y_hat")
        yl = float(yh.gather(1, y[:, None]).min()) if yh is not None else float("nan")
        nneg = int((yh.gather(1, y[:, None]) <= 0).sum()) if yh is not None else -1
        print(f"step {i:2d} loss {float(loss):.6f} lyap {float(pl['scalars'][0]):.6f} ode "
              f"{float(pl['loss_ode']) if 'loss_ode' in pl else float('nan'):.6f} min y_hat[label] {yl:.3e} (<= 0: {nneg}) "
              f"ms {dt:7.2f} stats {st} status_word {None if sw is None else int(sw[0])} skipped {sk}{flag}",
              flush=True)
    gs.close()


if __name__ == "__main__":
    if "--large" in sys.argv:                 # configs[4]'s shape: B=1024 x S=1024
        run("dopri5", steps=8, B=1024, S=1024)
    else:
        run("dopri5")
