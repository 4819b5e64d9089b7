#!/bin/bash
# round 4, pass j: PMC of the throughput kernels (fan-out fwd/bwd, cert fwd/final): MFMA-busy,
# wave issue/wait breakdown and the clock (GRBM_GUI_ACTIVE / duration), one pass per counter set
set -u
O=$PWD/gpurun_out/r04j; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/probes/tp_pmc.py > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_a -o run -- python $R/tools/probes/tp_pmc.py > $O/pmc_a.log 2>&1 || { echo pmc_a failed; tail $O/pmc_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT --output-format csv -d $O/pmc_b -o run -- python $R/tools/probes/tp_pmc.py > $O/pmc_b.log 2>&1 || { echo pmc_b failed; tail $O/pmc_b.log; exit 1; }
echo done
