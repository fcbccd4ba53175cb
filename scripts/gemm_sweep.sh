#!/bin/bash
# Large-tile GEMM timing experiments: pipeline variants x (full / no-MFMA / no-DMA).
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for pipe in ${PIPES:-0 1}; do
  for d in ${DBGS:-0 1 2}; do
    echo "== MFL_GB_PIPE=$pipe MFL_GB_DEBUG=$d"
    BIG_ONLY=1 MFL_GB_PIPE=$pipe MFL_GB_DEBUG=$d timeout -k 10 120 python scripts/gemm_micro.py || exit $?
  done
done
