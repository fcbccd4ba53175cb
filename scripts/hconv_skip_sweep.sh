#!/bin/bash
# halo conv per stage in the co-located regime (MFL_HCONV_SKIP / MFL_HCONV)
set -o pipefail
out=$1
run() {
  echo "=== $1" >> "$out"
  env $1 timeout -k 10 200 python scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "G=8" >> "$out"
}
for rep in 1 2 3; do
  run "MFL_HCONV_SKIP="


  run "MFL_HCONV_SKIP=4,32"
  run "MFL_HCONV_SKIP=4"
  run "MFL_HCONV=0"
done
