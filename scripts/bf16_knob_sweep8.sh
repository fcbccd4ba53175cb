#!/bin/bash
# bf16 option, 8 co-located learners (probe): BASE vs env variants, 3 repeats
set -o pipefail
out=$1; shift
for rep in 1 2 3; do
  for v in "BASE=1" "$@"; do
    echo "=== $v" >> "$out"
    env $v timeout -k 10 200 python scripts/multi_learner_probe.py --groups 8 --updates 256 --dtype bf16 2>&1 | grep "G=8" >> "$out"
  done
done
