#!/bin/bash
# r05ak: the bench's captured step (4 placement trials) as a node / edge list (HIP graph API) and a
# kernel trace of its replays: where a kernel starts later than its last graph predecessor ends
set -o pipefail
O=gpurun_out/${TAG:-r05ak}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
  python3 -u tools/probes/graph_dot_probe.py 4 40 > $O/dot.log 2>&1
