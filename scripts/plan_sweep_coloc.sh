#!/bin/bash
# Co-located (8 learners) step time under paired-backward plan overrides
# (MFL_C32_PLANS="mode,h,c,co,r,stride,splits", conv32.hip plan_overrides).
set -o pipefail
out=$1
run() {
  echo "=== $1" >> "$out"
  MFL_C32_PLANS="$1" timeout -k 10 200 python scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "G=8" >> "$out"
}
for rep in 1 2; do
run ""
for s in 8 16 32; do run "2,32,64,64,3,1,$s"; done
for s in 4 14; do run "2,16,128,128,3,1,$s"; done
for s in 1 4; do run "2,8,256,256,3,1,$s"; done
for s in 2 8; do run "1,4,512,512,3,1,$s"; done
for s in 2 8; do run "1,8,256,256,3,1,$s"; done
for s in 1 4; do run "1,16,128,128,3,1,$s"; done
done
