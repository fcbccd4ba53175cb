#!/bin/bash
# PMC passes over one throughput-regime conv kernel (scripts/tconv_check.cpp
# profile mode): pmc_tconv.sh <batch> <shape> <w|d> <cfg> <splits> <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/pmc_tconv/$6; mkdir -p $O
export TMPDIR=/tmp
B=$R/build/bench/tconv_check
A="$1 20 $2 0 $3 $4 $5"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1 -o run -- $B $A > $O/p1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p2 -o run -- $B $A > $O/p2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d $O/p3 -o run -- $B $A > $O/p3.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.txt
cat $O/summary.txt
