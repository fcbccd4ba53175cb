#!/bin/bash
# Whole-step PMC passes over the single-learner fp32 ResNet-18 step
# (scripts/step_prof.py): HBM bytes (FETCH_SIZE / WRITE_SIZE), L2 hit
# rate, MFMA / VALU / LDS instruction counts -- one rocprofv3 run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/pmc_step; mkdir -p $O
export PYTHONPATH=$R
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $O/p1 -o run -- python3 $R/scripts/step_prof.py --steps 16 --warmup 8 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --kernel-trace --output-format csv -d $O/p2 -o run -- python3 $R/scripts/step_prof.py --steps 16 --warmup 8 > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p3 -o run -- python3 $R/scripts/step_prof.py --steps 16 --warmup 8 > $O/p3.log 2>&1 || exit $?
ls -R $O | head -30
