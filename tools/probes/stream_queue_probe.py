"""Which hardware queue does each new HIP stream get?  (tools/probes; not a test.)  Makes 12 dedicated
streams (fiode_amd.streams.new_stream; priorities 0 and -1 interleaved as noted), launches one small
torch kernel on each in creation order, synchronising between launches; run it under
`rocprofv3 --kernel-trace` and read Queue_Id per launch (tools/probes prints the creation order)."""
import sys

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2] / "fi-ode_amd"))
from fiode_amd.streams import new_stream  # noqa: E402

dev = torch.device("cuda:0")
x = torch.zeros(1024, device=dev)
prios = [0] * 8 + [-1, 0, -1, 0]
streams = [new_stream(dev, p) for p in prios]
for i, (s, p) in enumerate(zip(streams, prios)):
    with torch.cuda.stream(s):
        x.add_(float(i + 1))        # the i-th launch of vectorized_elementwise_kernel
    torch.cuda.synchronize()
    print(i, "priority", p, "stream", hex(s.cuda_stream), flush=True)
