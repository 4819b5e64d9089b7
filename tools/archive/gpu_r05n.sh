#!/bin/bash
# round 5, pass n: the tree bisection (qp_bisect_tree) -- bit identity of the train_ode solve against
# the previous commit's library, the solve tests, solve timings, per-eval phases, step A/B
set -u
R=$PWD; O=$R/gpurun_out/r05n; mkdir -p $O
FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/ab_odetrain.py $O/base.pt > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
timeout -k 10 120 python -u tools/ab_odetrain.py $O/new.pt >> $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
python tools/ab_odetrain.py --cmp $O/base.pt $O/new.pt >> $O/ab.log 2>&1; echo "cmp rc=$?" >> $O/ab.log
grep -c identical $O/ab.log; grep DIFFER $O/ab.log | head; tail -1 $O/ab.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_odetrain.py tests/test_gpu_odetrain_dp.py \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/solve_ab.py > $O/solve_base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probes/solve_ab.py > $O/solve_new_$r.log 2>&1 || exit 1
done
for f in $O/solve_*.log; do echo "== $f"; grep -v "amdgpu.ids" $f; done
timeout -k 10 120 python -u tools/ot_probe.py > $O/ot_probe.log 2>&1 || { tail $O/ot_probe.log; exit 1; }
grep "per eval" $O/ot_probe.log
timeout -k 10 120 python -u tools/probes/odp_probe.py > $O/odp_probe.log 2>&1 || { tail $O/odp_probe.log; exit 1; }
tail -12 $O/odp_probe.log
bash tools/gpu_lib_ab.sh r05n/ab 3 || exit 1
