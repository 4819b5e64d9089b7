"""Does the hipGraph executor release a captured graph's work by dependency level? (not a test)

python tools/probes/graph_level_probe.py  ->  one JSON line of replay times (us)

Two independent branches forked from one stream inside a capture: branch L = one long kernel
(torch.cuda._sleep, ~S us) on a side stream, branch C = a chain of N small dependent kernels on the
capture stream.  With every branch free to run, a replay takes ~max(S, N * t_small); if the executor
holds each level until the previous one has finished, ~S + N * t_small.  Measured for N = 1, 8, 32
against each branch alone.
"""
import json
import time

import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
x = torch.zeros(1 << 16, device=dev)
side = torch.cuda.Stream(dev)
SLEEP = 200_000          # cycles of torch.cuda._sleep


def build(n_chain, long_branch=True, chain=True, side_parts=1):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        main = torch.cuda.current_stream()
        if long_branch:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(side_parts):          # the side branch as a chain of side_parts kernels
                    torch.cuda._sleep(SLEEP // side_parts)
        if chain:
            for _ in range(n_chain):
                x.add_(1.0)
        if long_branch:
            main.wait_stream(side)
    return g


def clock(g, n=50):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


res = {"long_only": clock(build(0, True, False))}
for n in (1, 8, 32):
    res[f"chain{n}_only"] = clock(build(n, False, True))
    res[f"both{n}"] = clock(build(n, True, True))
res["side12_only"] = clock(build(0, True, False, side_parts=12))
for n in (8, 32):
    res[f"side12_both{n}"] = clock(build(n, True, True, side_parts=12))
# the remedy to test: the two branches as two graphs launched on two streams (each replayed as a
# unit on its own stream, joined by an event)
g_long, g_chain = build(0, True, False, side_parts=12), build(32, False, True)
s2 = torch.cuda.Stream(dev)


def two_graphs(n=50):
    main = torch.cuda.current_stream()

    def once():
        s2.wait_stream(main)
        with torch.cuda.stream(s2):
            g_long.replay()
        g_chain.replay()
        main.wait_stream(s2)
    for _ in range(5):
        once()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        once()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


res["two_graphs_side12_chain32"] = two_graphs()
print(json.dumps(res), flush=True)
