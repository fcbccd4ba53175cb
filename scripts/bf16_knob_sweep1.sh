#!/bin/bash
# bf16 option, ONE learner (probe) under env knobs; each arg one variant
set -o pipefail
out=$1; shift
for rep in 1 2; do
  for v in "BASE=1" "$@"; do
    echo "=== $v" >> "$out"
    env $v timeout -k 10 200 python scripts/multi_learner_probe.py --groups 1 --updates 512 --dtype bf16 2>&1 | grep "G=1" >> "$out"
  done
done
