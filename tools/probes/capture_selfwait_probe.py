"""Which stream-capture event patterns crash this ROCm runtime at capture end?  (tools/probes; not a
test -- VERDICT r05 item 2, the capture_end SIGSEGV.)  Each case in a child process (rc -11 = SIGSEGV).

  self_wait     s records e, then s waits on e (a wait on an event last recorded on the same stream)
  self_wait_k   the same with a kernel between the record and the wait
  relay         side waits on e (recorded on main), records e2 with no kernel of its own, main waits on e2
  relay_work    relay, then later side waits on main again and runs a kernel, joined back
  wait_stream_self   torch's s.wait_stream(s)
"""
import subprocess
import sys

CASE = r'''
import sys, torch
case = sys.argv[1]
dev = torch.device("cuda:0")
x = torch.zeros(1 << 16, device=dev)
main_s = torch.cuda.Stream(dev)
side = torch.cuda.Stream(dev)
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, stream=main_s, capture_error_mode="thread_local"):
        cur = torch.cuda.current_stream()
        x.add_(1.0)
        if case in ("self_wait", "self_wait_k"):
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                x.mul_(2.0)
                e = torch.cuda.Event(); e.record(side)
                if case == "self_wait_k":
                    x.mul_(2.0)
                side.wait_event(e)
                x.add_(1.0)
            cur.wait_stream(side)
        elif case in ("relay", "relay_work"):
            e = torch.cuda.Event(); e.record(cur)
            side.wait_event(e)
            e2 = torch.cuda.Event(); e2.record(side)
            cur.wait_event(e2)
            x.add_(3.0)
            if case == "relay_work":
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    x.mul_(2.0)
                cur.wait_stream(side)
        elif case == "wait_stream_self":
            cur.wait_stream(cur)
            x.add_(2.0)
        x.add_(5.0)
    g.replay()
    torch.cuda.synchronize()
    print("ok", float(x[0]))
except Exception as ex:
    print("python error:", type(ex).__name__, str(ex).splitlines()[0])
'''


def main():
    for case in ("relay", "relay_work", "wait_stream_self", "self_wait_k", "self_wait"):
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", CASE, case], capture_output=True, text=True,
                           timeout=120)
        out = (r.stdout.strip().splitlines() or [""])[-1]
        print(f"{case:18s} exit {r.returncode:4d}  {out}", flush=True)


if __name__ == "__main__":
    main()
