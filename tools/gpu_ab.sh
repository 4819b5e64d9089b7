#!/bin/bash
# train_ode A/B pass: GPU tests of the solve, A/B bit identity against a previous
# build (tools/libfiode_base.so: `git archive <rev> fi-ode_amd/csrc include | tar -x -C /tmp/base`
# and `make -C /tmp/base/fi-ode_amd/csrc OUT=$PWD/tools/libfiode_base.so OBJDIR=/tmp/base/build`),
# phase probe, bench.  Stops at the first failing step.
set -u
O=gpurun_out/${1:-spec}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python tools/ab_odetrain.py $O/ab_base.pt > $O/ab.log 2>&1 || { echo "ab base rc=$?"; exit 1; }
timeout -k 10 120 python tools/ab_odetrain.py $O/ab_new.pt >> $O/ab.log 2>&1 || { echo "ab new rc=$?"; exit 1; }
python tools/ab_odetrain.py --cmp $O/ab_base.pt $O/ab_new.pt >> $O/ab.log 2>&1; echo "ab cmp rc=$?"; cat $O/ab.log
timeout -k 10 180 python tools/ot_probe.py > $O/ot_probe.log 2>&1 || { echo "ot_probe rc=$?"; exit 1; }
cat $O/ot_probe.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['per_kernel_ms'], d.get('dopri5_train_step'))"
