#!/bin/bash
# One command under several settings of one environment variable, alternating
# the settings in each repeat on one box:
#   scripts/env_sweep.sh <log> <reps> <VAR> "<v1> <v2> ..." <command...>
# (an empty value "-" leaves the variable unset)
set -o pipefail
log=$1; reps=$2; var=$3; vals=$4; shift 4
for r in $(seq 1 "$reps"); do
  for v in $vals; do
    echo "=== $var=$v rep $r" >> "$log"
    if [ "$v" = "-" ]; then
      timeout -k 10 300 "$@" >> "$log" 2>&1 || { echo "FAILED $v $r" >> "$log"; exit 1; }
    else
      env "$var=$v" timeout -k 10 300 "$@" >> "$log" 2>&1 || { echo "FAILED $v $r" >> "$log"; exit 1; }
    fi
  done
done
