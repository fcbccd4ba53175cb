#!/bin/bash
set -o pipefail
out=$1
for r in 1 2; do
  for p in none default; do
    echo "=== $p rep $r" >> "$out"
    if [ "$p" = none ]; then MFL_COLOC_PLANS="" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 >> "$out" 2>&1 || exit 1
    else timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 >> "$out" 2>&1 || exit 1; fi
  done
done
