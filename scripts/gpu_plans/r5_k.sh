set -o pipefail
# round 5: driver collective GPU tests; GEMM epilogue read hoist: BERT/GEMM tests, bench + kernel trace
O=gpurun_out/r5k; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_driver_collective_gpu.py > $O/driver.log 2>&1 || { tail -30 $O/driver.log; exit 1; }
tail -2 $O/driver.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bert_gpu.py tests/test_gemm_gpu.py > $O/gemm.log 2>&1 || { tail -30 $O/gemm.log; exit 1; }
tail -2 $O/gemm.log
TESTS=0 BERT_ARGS="--steps 2 --warmup 1" bash scripts/bert_prof.sh && cp -r gpurun_out/bert_prof $O/ && cp gpurun_out/bert_bench.log $O/
