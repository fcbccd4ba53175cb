#!/bin/bash
# ResNet-18 step time vs the paired conv backward's plans (env knobs).
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
while read -r env; do
  [ -z "$env" ] && continue
  r=$(env $env timeout -k 10 120 python bench.py --local-epochs 1 --steps 2 --warmup 1 --train-size 16384 --no-eval 2>&1 | grep '^\[bench\] round 3') || exit 1
  echo "$env :: $r"
done <<< "${CFGS:-MFL_CONV_PAIR=1
MFL_PAIR_WGRAD_TARGET=256
MFL_PAIR_WGRAD_TARGET=128
MFL_PAIR_DGRAD_SPLIT_DIV=2
MFL_PAIR_WGRAD_TARGET=1024
MFL_CONV_PAIR=1}"
