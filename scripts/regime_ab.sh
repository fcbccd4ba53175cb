#!/bin/bash
# bench A/B of one co-located regime knob: "$@" = env assignment for variant B
set -o pipefail
out=$1; shift
for r in 1 2; do
  echo "=== A rep $r" >> "$out"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 >> "$out" 2>&1 || exit 1
  echo "=== B($*) rep $r" >> "$out"
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 >> "$out" 2>&1 || exit 1
done
