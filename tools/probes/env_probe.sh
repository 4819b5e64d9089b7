# Step time under HIP graph-executor queue settings, alternated A B A B ... (not a test).
# usage (via gpurun): bash tools/probes/env_probe.sh
set -u
mkdir -p gpurun_out/env
for round in 1 2 3; do
  for v in "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=3" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
    tag=$(echo "$v" | tr '=' '_')
    env $v timeout -k 10 150 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/env/$tag.json 2> gpurun_out/env/$tag.err || { echo "$v failed"; exit 1; }
    echo "$round $v $(python -c "import json;d=json.load(open('gpurun_out/env/$tag.json'));print(d['ms_per_step'])")"
  done
done
