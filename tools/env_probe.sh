set -u
mkdir -p gpurun_out/env
for v in "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=64"; do
  tag=$(echo "x$v" | tr '=' '_')
  env $v timeout -k 10 150 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/env/$tag.json 2> gpurun_out/env/$tag.err || { echo "$v failed"; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/env/$tag.json'));print(d['value'], d['ms_per_step'])")"
done
