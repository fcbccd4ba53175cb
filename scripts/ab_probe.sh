#!/bin/bash
# two kernel builds (build/ab/_ops_base.so vs the tree's) on the co-located
# and one-learner ResNet probe, alternating
set -o pipefail
log=$1; reps=$2; shift 2
so=$(ls metisfl_amd/_ops*.so); cp "$so" /tmp/_ops_new.so
for r in $(seq 1 "$reps"); do
  for v in base new; do
    if [ $v = base ]; then cp build/ab/_ops_base.so "$so"; else cp /tmp/_ops_new.so "$so"; fi
    echo "=== $v rep $r" >> "$log"
    timeout -k 10 300 python scripts/multi_learner_probe.py --groups 8 --updates 256 "$@" 2>&1 | grep "G=" >> "$log" || { cp /tmp/_ops_new.so "$so"; exit 1; }
    timeout -k 10 300 python scripts/multi_learner_probe.py --groups 1 --updates 512 "$@" 2>&1 | grep "G=" >> "$log" || { cp /tmp/_ops_new.so "$so"; exit 1; }
  done
done
cp /tmp/_ops_new.so "$so"
