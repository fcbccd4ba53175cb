#!/bin/bash
# Conv plan sweep: short benches under different plan knobs (env vars read by
# plan_conv_gemm / plan_conv_wgrad).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
ARGS="--local-epochs 1 --steps 2 --warmup 1 --train-size 16384 --test-size 1024"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS > gpurun_out/sweep/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"train_ms_mean": [0-9.]*' gpurun_out/sweep/$name.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
}
run base
run m2 MFL_CONV_MIN_KSTEPS=2
run m3 MFL_CONV_MIN_KSTEPS=3
run t512_m2 MFL_CONV_TARGET_BLOCKS=512 MFL_CONV_MIN_KSTEPS=2
run t128 MFL_CONV_TARGET_BLOCKS=128
