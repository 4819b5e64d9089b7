"""Does this ROCm runtime survive a hipGraph capture that ends with a forked stream not joined back
into the origin stream?  (tools/probes; not a test -- VERDICT r05 item 2, the r05ae capture_end
SIGSEGV.)  CUDA's contract is an error (cudaErrorStreamCaptureUnjoined) from EndCapture.  Each case
runs in a child process; the parent prints the child's exit status (-11 = SIGSEGV).

  joined     fork s1 from the capture stream, work on s1, join it back        (the product's form)
  unjoined   the same without the join                                         (a tap node whose
             side-stream branch nothing on the capture stream waits for)
  recapture  capture / replay / re-capture on FRESH side streams with the old graph dropped first
             (GraphTrainStep._select_placement's trial loop), joined
"""
import subprocess
import sys

CASE = r'''
import sys, torch
case = sys.argv[1]
dev = torch.device("cuda:0")
x = torch.zeros(1 << 16, device=dev)
def cap(side, join):
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cs, capture_error_mode="thread_local"):
        x.add_(1.0)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x.mul_(2.0)
        if join:
            torch.cuda.current_stream().wait_stream(side)
        x.add_(3.0)
    return g
try:
    if case == "joined":
        g = cap(torch.cuda.Stream(dev), True)
        g.replay()
    elif case == "unjoined":
        g = cap(torch.cuda.Stream(dev), False)
        g.replay()
    elif case == "recapture":
        g = None
        for t in range(6):
            g = None                      # the previous trial's graph dropped before the new capture
            g = cap(torch.cuda.Stream(dev), True)
            for _ in range(3):
                g.replay()
    torch.cuda.synchronize()
    print("ok", float(x[0]))
except Exception as e:
    print("python error:", type(e).__name__, str(e).splitlines()[0])
'''


def main():
    for case in ("joined", "recapture", "unjoined"):
        r = subprocess.run([sys.executable, "-c", CASE, case], capture_output=True, text=True, timeout=120)
        out = (r.stdout.strip().splitlines() or [""])[-1]
        err = [ln for ln in r.stderr.splitlines() if "amdgpu.ids" not in ln][-2:]
        print(f"{case:10s} exit {r.returncode:4d}  {out}  {' | '.join(err)}", flush=True)


if __name__ == "__main__":
    main()
