#!/bin/bash
# round 4, pass ah: MFMA-busy of the throughput kernels (bench shape, configs[4] shape, T=40 image)
set -u
O=$PWD/gpurun_out/r04ah; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python $R/tools/probes/tp_pmc.py > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
cd $R
python tools/pmc_busy.py $O/pmc/run_counter_collection.csv | tee $O/busy.txt
