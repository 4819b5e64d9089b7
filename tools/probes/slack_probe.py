"""Critical-path probe of the replayed configs[1] step (not a test): a ~200 us GPU spin is
inserted in front of one part of the step (on whatever stream that part runs), and the growth of
the hipGraph step time tells whether that part is on the critical path (growth ~ 200 us) or has
slack (growth ~ 0).

python tools/probes/slack_probe.py  ->  one JSON line: ms per step per variant (captures picked from 4
placement trials, as bench.py does; a spin in front of a call made k times per step adds k x 200 us
when every one of them is on the critical path)
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import cayley as CY, lyapunov as LY, ops  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def calib():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    a.record()
    torch.cuda._sleep(1_000_000)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1_000_000


MS_PER_CYCLE = calib()
SPIN = int(0.2 / MS_PER_CYCLE)     # cycles for ~200 us


def step_ms(steps=40):
    mod = bench.build_module(dev, train_ode=True)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    gs = GraphTrainStep(mod, opt, x, y, placement_trials=4)
    for _ in range(5):
        gs.step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        gs.step()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / steps * 1e3, 4)


def spin_before(owner, name, once_per_step=True):
    orig = getattr(owner, name)

    def wrapped(*a, **k):
        torch.cuda._sleep(SPIN)
        return orig(*a, **k)
    setattr(owner, name, wrapped)
    return lambda: setattr(owner, name, orig)


variants = [
    ("baseline", None),
    ("conv1_input_transform (step start)", (ops, "sconv_rfft2_nchw")),
    ("conv1_irfft2_qx", (ops, "sconv_irfft2_qx")),
    ("head_out (head fwd end)", (ops, "head_out")),
    ("linear_map_fwd (side streams 1-2)", (CY.CayleyLinear, "effective_weight")),
    ("dyn_map_fwd (side stream 3)", (__import__("fiode_amd.dynamics", fromlist=["x"]), "cayley_scaled")),
    ("lyap_step (fan-out)", (ops, "lyap_step")),
    ("odetrain_fwd (ode stream)", (ops, "odetrain_forward")),
    ("odetrain_bwd_x", (ops, "odetrain_backward_x")),
    ("odetrain_bwd_weights (tap, side)", (ops, "odetrain_backward_weights")),
    ("head_out_backward_gs (head bwd start)", (ops, "head_out_backward_gs")),
    ("conv_map_bwd (layer streams, x4)", (ops, "spectral_cayley_backward")),
    ("conv_map_refresh (layer streams, x4)", (CY.CayleyConv, "refresh_map")),
    ("dense_map_bwd (x3)", (CY, "_dense_backward")),
]
if len(sys.argv) > 1 and sys.argv[1] == "lyap_curve":
    variants = [("baseline", None)]
    for us in (10, 30, 60, 120, 200, 300):
        variants.append((f"lyap spin {us} us", (ops, "lyap_step", us)))
res = {}
for name, tgt in variants:
    if tgt is not None and len(tgt) == 3:
        SPIN = int(tgt[2] * 1e-3 / MS_PER_CYCLE)
        tgt = tgt[:2]
    undo = spin_before(*tgt) if tgt else (lambda: None)
    try:
        res[name] = step_ms()
    finally:
        undo()
    print(name, res[name], file=sys.stderr, flush=True)
print(json.dumps({"spin_us": 200, **res}), flush=True)
