#!/bin/bash
# ResNet-18 step time vs the conv wgrad split-K plan (MFL_WGRAD_TARGET_BLOCKS /
# MFL_WGRAD_MIN_KSTEPS): fewer slices = fewer memory-side fp32 atomic bytes.
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for cfg in ${CFGS:-"512 8" "256 8" "128 8" "512 16" "512 32" "64 8"}; do
  set -- $cfg
  r=$(MFL_WGRAD_TARGET_BLOCKS=$1 MFL_WGRAD_MIN_KSTEPS=$2 timeout -k 10 120 python bench.py --local-epochs 1 --steps 2 --warmup 1 --train-size 16384 --no-eval 2>&1 | grep '^\[bench\] round' | tail -1) || exit 1
  echo "target=$1 min_ksteps=$2 $r"
done
