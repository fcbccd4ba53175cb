#!/bin/bash
# Conv timing experiment: per-layer graph-replay timings of conv_micro.py with
# MFL_CONV_DEBUG = 0 (normal), 1 (no MFMA), 2 (no DMA), 3 (neither).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/dbg
for m in 0 1 2 3; do
  echo "== MFL_CONV_DEBUG=$m"
  cd $R && MFL_CONV_DEBUG=$m PYTHONPATH=$R timeout -k 10 240 python3 $R/scripts/conv_micro.py 50 || exit $?
done
