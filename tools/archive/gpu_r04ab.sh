#!/bin/bash
# round 4, pass ab: the captured one-graph step under the HIP runtime's graph-launch settings
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE, DEBUG_HIP_GRAPH_BATCH_SIZE); default first and last
set -u
O=$PWD/gpurun_out/r04ab; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-configs --steps 40 --warmup 10 > $O/$tag.json 2>$O/$tag.err \
    || { echo "$tag failed rc=$?"; tail -3 $O/$tag.err; return 1; }
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
run default0 FIODE_X=0 &&
run pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 &&
run bs8 DEBUG_HIP_GRAPH_BATCH_SIZE=8 &&
run bs64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 &&
run default1 FIODE_X=0 && echo done
