#!/bin/bash
# Second co-located plan sweep, on top of the co-located defaults
set -o pipefail
out=$1
B="1,16,128,128,3,1,1;1,8,256,256,3,1,2"
run() {
  echo "=== ${1:-base}" >> "$out"
  MFL_C32_PLANS="$B${1:+;$1}" timeout -k 10 200 python scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "G=8" >> "$out"
}
for rep in 1 2; do
run ""
run "2,32,64,128,3,2,7"; run "2,32,64,128,3,2,28"; run "2,32,64,128,1,2,26"
run "1,16,128,256,3,2,1"; run "1,16,128,256,3,2,2"; run "2,16,128,256,3,2,4"; run "2,16,128,256,1,2,7"
run "1,8,256,512,3,2,2"; run "2,8,256,512,1,2,2"; run "1,8,256,512,1,2,1"
run "0,16,128,256,3,2,2"; run "0,8,256,512,3,2,2"
done
