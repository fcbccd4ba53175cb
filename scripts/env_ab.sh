#!/bin/bash
# A/B of one environment knob under the same command, alternating arms on one
# box (same-process-order repeats):
#   scripts/env_ab.sh <log> <reps> <VAR=a> <VAR=b> <command...>
set -o pipefail
log=$1; reps=$2; a=$3; b=$4; shift 4
for r in $(seq 1 "$reps"); do
  for v in "$a" "$b"; do
    echo "=== $v rep $r" >> "$log"
    env "$v" timeout -k 10 300 "$@" >> "$log" 2>&1 || { echo "FAILED $v $r" >> "$log"; exit 1; }
  done
done
