set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tconv_gpu.py "tests/test_fp32_gpu.py::test_fp32_resnet18_step_matches_torch_nn" tests/test_graph_k8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 4 8 --updates 256 --tconv 0 > $O/ml_t0.log 2>&1 && \
timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 4 8 --updates 256 --tconv 1 > $O/ml_t1.log 2>&1 && \
timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 4 8 --updates 256 --tconv 0 > $O/ml_t0b.log 2>&1 && \
timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 4 8 --updates 256 --tconv 1 > $O/ml_t1b.log 2>&1
grep -h "ms per" $O/ml_*.log
