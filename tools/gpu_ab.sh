set -u
export TMPDIR=/tmp
O=gpurun_out/ab2; mkdir -p $O
FIODE_LIB=$PWD/tools/libfiode_ref.so timeout -k 10 120 python tools/ab_odetrain.py $O/ref.pt > $O/ref.log 2>&1 || { echo ref failed; exit 1; }
timeout -k 10 120 python tools/ab_odetrain.py $O/new.pt > $O/new.log 2>&1 || { echo new failed; tail $O/new.log; exit 1; }
python tools/ab_odetrain.py --cmp $O/ref.pt $O/new.pt
timeout -k 10 300 python -u -m pytest tests/test_gpu_odetrain.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo pytest rc=$?; tail -3 $O/pytest.log
timeout -k 10 150 python tools/probes/kexit_probe.py > $O/kexit.log 2>&1; tail -4 $O/kexit.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; echo bench rc=$?
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['per_kernel_ms'], d['lyapunov_only_step'])"
timeout -k 10 150 python tools/ot_probe.py > $O/otprobe.log 2>&1; grep -v Warn $O/otprobe.log | tail -8
