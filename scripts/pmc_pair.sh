#!/bin/bash
# PMC passes over the paired conv32 backward (scripts/hdgrad_bench.py --eager):
# one rocprofv3 run per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/pmc_pair; mkdir -p $O
export PYTHONPATH=$R
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/p1 -o run -- python3 $R/scripts/hdgrad_bench.py --eager 5 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d $O/p2 -o run -- python3 $R/scripts/hdgrad_bench.py --eager 5 > $O/p2.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $(find $O -name "*counter_collection.csv") --filter=pair > $O/summary.txt
cat $O/summary.txt
