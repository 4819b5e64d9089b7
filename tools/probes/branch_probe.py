"""Do independent captured branches run concurrently under hipGraph replay? (not a test)
Times the 4096->512 and 512->512 Cayley maps (each a ~200 us latency chain) captured alone, and
both captured on two side streams of one graph; concurrent branches give ~max, serial ones ~sum.

python tools/probes/branch_probe.py  ->  one JSON line of us per replay
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.cayley import CayleyLinear  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def replay_us(fn, reps=40):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 1)


mod = bench.build_module(dev, train_ode=True)
lins = [m for m in mod.init_coordinates.modules() if isinstance(m, CayleyLinear)]
side = [torch.cuda.Stream(dev) for _ in range(3)]


def on_streams(ms):
    def fn():
        main = torch.cuda.current_stream()
        outs = []
        for m, st in zip(ms, side):
            st.wait_stream(main)
            with torch.cuda.stream(st), torch.no_grad():
                outs.append(m.effective_weight())
        for st in side[:len(ms)]:
            main.wait_stream(st)
        return outs
    return fn


res = {"lin0": replay_us(on_streams([lins[0]])), "lin1": replay_us(on_streams([lins[1]])),
       "lin0+lin1": replay_us(on_streams([lins[0], lins[1]])),
       "lin0+lin1+lin2": replay_us(on_streams([lins[0], lins[1], lins[2]]))}
print(json.dumps(res), flush=True)
