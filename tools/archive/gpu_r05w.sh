#!/bin/bash
# round 5, pass v: padded complex pivot rows of gj.h: inverse / map tests, timings
# against the previous commit, and the LDS bank-conflict PMC pass
set -u
R=$PWD; O=$R/gpurun_out/r05w; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cayley.py \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  FIODE_LIB=tools/libfiode_base.so timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probes/spec_probe.py > $O/new_$r.log 2>&1 || exit 1
done
for f in $O/base_1.log $O/new_1.log $O/base_2.log $O/new_2.log; do echo "== $f"; grep -v "amdgpu.ids\|^lib" $f; done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc -o run -- python $R/tools/probes/spec_probe.py > $O/pmc.log 2>&1 || { echo "pmc failed rc=$?"; tail $O/pmc.log; exit 1; }
echo pmc done
