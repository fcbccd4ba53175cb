#!/bin/bash
# BERT-base: GPU tests, short federation bench + rocprofv3 kernel statistics.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -m pytest tests/test_bert_gpu.py -q -x -m gpu > gpurun_out/bert_tests.log 2>&1 || { tail -20 gpurun_out/bert_tests.log; exit 1; }
  tail -2 gpurun_out/bert_tests.log
fi
timeout -k 10 600 python benchmarks/bert_bench.py ${BERT_ARGS:---steps 2 --warmup 1} > gpurun_out/bert_bench.log 2>&1 || exit $?
tail -1 gpurun_out/bert_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bert_prof -o run -- python3 $R/benchmarks/bert_bench.py --steps 1 --warmup 0 --local-steps 10 > $R/gpurun_out/bert_prof.log 2>&1
