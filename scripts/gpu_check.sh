#!/bin/bash
# GPU-box validation: numerics tests, a short bench and a rocprofv3 kernel
# profile.  Stops at the first crash-class exit (abort/segv/timeout/kill).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_resnet_gpu.py"}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest $TESTS -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if crash $rc; then echo "stopping after crash-class exit"; exit $rc; fi

if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---local-epochs 1 --steps 2 --warmup 1} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/bench.log
  if crash $rc; then exit $rc; fi
fi

if [ "${PROF:-1}" = "1" ]; then
  cd /tmp
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---local-epochs 1 --steps 1 --warmup 0 --train-size 8192 --test-size 1024} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "prof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
  cd "$GRAFT_REPO_ROOT"
fi
exit 0
