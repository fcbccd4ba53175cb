#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/pmc
export PYTHONPATH=$R
timeout -k 10 200 python scripts/conv_micro.py 50 > gpurun_out/pmc/micro.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p1 -o run -- python3 $R/scripts/conv_micro.py 5 > $R/gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p2 -o run -- python3 $R/scripts/conv_micro.py 5 > $R/gpurun_out/pmc/p2.log 2>&1
echo done
