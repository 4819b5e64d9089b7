"""Which stream layout of the Cayley-map prefetch gives the shortest replayed configs[1] step
(not a test).  The hipGraph executor maps the captured streams onto the process's hardware
queues (GPU_MAX_HW_QUEUES = 4 on the pool's boxes), so independent branches can be serialized;
each variant assigns the 11 maps (4 conv, 3 linear, dynamics) to side streams differently.

python tools/probes/stream_probe.py  ->  one JSON line of ms per step per variant
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import lyapunov as LY  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def step_ms(mod, steps=30):
    opt = mod.configure_optimizers(capturable=True)[0][0]
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    gs = GraphTrainStep(mod, opt, x, y)
    for _ in range(5):
        gs.step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        gs.step()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / steps * 1e3, 4)


def layout(conv, lin, dyn, nstreams=4):
    """conv / lin: list of stream indices per layer (None = not prefetched), dyn: index or None."""
    def pf(self, device):
        if self._side_streams is None or len(self._side_streams) < nstreams:
            self._side_streams = [torch.cuda.Stream(device) for _ in range(nstreams)]
        s = self._side_streams
        convs, lins = [], []
        for m in self.init_coordinates.modules():
            if hasattr(m, "prefetch") and m is not self.dyn_fun:
                (convs if hasattr(m, "spectral_weight") else lins).append(m)
        order = [("c", i) for i in range(len(convs))] + [("l", i) for i in range(len(lins))]
        for kind, i in order:
            si = (conv if kind == "c" else lin)[i]
            if si is not None:
                (convs if kind == "c" else lins)[i].prefetch(s[si])
        if dyn is not None:
            self.dyn_fun.prefetch(s[dyn])
    return pf


variants = {
    "current": None,
    "lin_on_conv_stream": layout([0, 0, 0, 0], [0, 0, 0], 3),
    "lin_big_own_rest_s0": layout([0, 0, 0, 0], [1, 0, 0], 0),
    "two_side_streams": layout([0, 0, 0, 0], [1, 1, 1], 1),
    "one_side_stream": layout([0, 0, 0, 0], [0, 0, 0], 0),
    "convs_split": layout([0, 1, 0, 1], [2, 3, 3], 3),
    "no_prefetch_lin": layout([0, 0, 0, 0], [None, None, None], 3),
}
from fiode_amd import cayley as CY  # noqa: E402
variants = {"current": None, "spec_bwd_main": "S", "dense_bwd_main": "D", "both_bwd_main": "SD",
            "current_2": None, "spec_bwd_main_2": "S", "dense_bwd_main_2": "D", "both_bwd_main_2": "SD"}
_unused = {"current": None,
            "lin2_dyn2": {"lin": [2, 2, 2], "dyn": 2},
            "current_again": None,
            "lin2_dyn3": {"lin": [2, 2, 2], "dyn": 3},
            "lin1_2_2_dyn3": {"lin": [1, 2, 2], "dyn": 3},
            "lin2_3_3_dyn3": {"lin": [2, 3, 3], "dyn": 3},
            "lin2_dyn_start": {"lin": [2, 2, 2], "dyn": -1},
            "lin2_dyn2_again": {"lin": [2, 2, 2], "dyn": 2}}
orig = LY.LyapunovLearning._prefetch_weights
res = {}
for name, pf in variants.items():
    mod = bench.build_module(dev, train_ode=True)
    CY.SPECTRAL_BWD_ON_MAIN = isinstance(pf, str) and "S" in pf
    CY.DENSE_BWD_ON_MAIN = isinstance(pf, str) and "D" in pf
    if isinstance(pf, str):
        pf = None
    if isinstance(pf, dict):
        mod.prefetch_schedule = pf
    else:
        LY.LyapunovLearning._prefetch_weights = pf if pf is not None else orig
    try:
        res[name] = step_ms(mod)
    except Exception as e:  # noqa: BLE001
        res[name] = f"failed: {str(e).splitlines()[0][:80]}"
    print(name, res[name], file=sys.stderr, flush=True)
    del mod
    torch.cuda.synchronize()
LY.LyapunovLearning._prefetch_weights = orig
print(json.dumps(res), flush=True)
