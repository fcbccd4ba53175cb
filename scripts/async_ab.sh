#!/bin/bash
set -o pipefail
out=$1
for r in 1 2; do
  for v in 1 0; do
    echo "=== MFL_ASYNC_HP=$v rep $r" >> "$out"
    MFL_ASYNC_HP=$v timeout -k 10 300 python benchmarks/async_bench.py >> "$out" 2>&1 || exit 1
  done
done
