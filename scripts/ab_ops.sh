#!/bin/bash
# A/B of two builds of the kernel extension on one box: alternates
# build/ab/_ops_base.so and the tree's _ops*.so under the same command.
#   scripts/ab_ops.sh <log> <reps> <command...>
set -o pipefail
log=$1; reps=$2; shift 2
so=$(ls metisfl_amd/_ops*.so)
cp "$so" build/ab/_ops_new.so
for r in $(seq 1 "$reps"); do
  for v in base new; do
    cp "build/ab/_ops_$v.so" "$so"
    echo "=== $v rep $r" >> "$log"
    timeout -k 10 300 "$@" >> "$log" 2>&1 || { echo "FAILED $v $r" >> "$log"; cp build/ab/_ops_new.so "$so"; exit 1; }
  done
done
cp build/ab/_ops_new.so "$so"
