"""Probe (not a test): a captured graph of K parallel branches, each on its own fresh stream (a chain
of a few small kernels), replayed 20 times -- the minimal shape of the training step's hipGraph.  The
parent runs one child per (GPU_MAX_HW_QUEUES, K) so a host fault in the runtime stays in its child
(rc 139 = SIGSEGV), with the native backtrace handler armed.

python tools/probes/hwq_branch_probe.py            (parent: the matrix)
python tools/probes/hwq_branch_probe.py child K    (one case, env from the parent)"""
import ctypes
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]


def child(k: int) -> None:
    ctypes.CDLL(str(ROOT / "tools" / "native" / "libsegv_bt.so"))
    import torch
    dev = torch.device("cuda:0")
    a = torch.ones(1 << 16, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream(dev), capture_error_mode="thread_local"):
        cur = torch.cuda.current_stream()
        outs = []
        for s in streams:
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                b = a
                for _ in range(4):
                    b = b * 1.0001 + 1.0
                outs.append(b)
        for s in streams:
            cur.wait_stream(s)
        tot = sum(outs)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    print(f"K={k} ok {float(tot[0]):.4f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
        sys.exit(0)
    for q in [a for a in sys.argv[1:]] or ("2", "4"):
        for k in (2, 3, 4, 6, 8, 12):
            env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
            p = subprocess.run([sys.executable, __file__, "child", str(k)], env=env, capture_output=True, text=True,
                               timeout=120)
            tail = (p.stdout.strip().splitlines() or [""])[-1]
            frames = [ln for ln in p.stderr.splitlines() if "libamdhip64" in ln][:3]
            print(f"GPU_MAX_HW_QUEUES={q} K={k}: rc {p.returncode} {tail} {' | '.join(frames)}", flush=True)
