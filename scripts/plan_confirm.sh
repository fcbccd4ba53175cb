#!/bin/bash
set -o pipefail
out=$1; shift
for rep in 1 2 3; do
  for p in "" "$@"; do
    echo "=== ${p:-base}" >> "$out"
    MFL_C32_PLANS="${BASEP}${p:+;$p}" timeout -k 10 200 python scripts/multi_learner_probe.py --groups 1 8 --updates 256 2>&1 | grep "G=" >> "$out"
  done
done
