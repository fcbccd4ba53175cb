#!/bin/bash
# A/B of the deferred community evaluation's stream (MFL_CE_STREAM) on one box
set -o pipefail
out=$1
for r in 1 2; do
  for k in plain prio cumask; do
    echo "=== $k rep $r" >> "$out"
    MFL_CE_STREAM=$k timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 >> "$out" 2>&1 || exit 1
  done
done
