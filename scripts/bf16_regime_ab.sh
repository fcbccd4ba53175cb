#!/bin/bash
# bf16 option: co-located regime split targets on / off, 1 / 2 / 4 / 8 learners
set -o pipefail
out=$1
for rep in 1 2; do
  for v in "MFL_COLOC_BF16_TARGETS=" "BASE=1"; do
    echo "=== $v" >> "$out"
    env "$v" timeout -k 10 300 python scripts/multi_learner_probe.py --groups 1 2 4 8 --updates 256 --dtype bf16 2>&1 | grep "G=" >> "$out"
  done
done
