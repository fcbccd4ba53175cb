set -o pipefail
O=gpurun_out/r5c; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/tconv_step_diff.py > $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 1; }
sort -g -k3 $O/diff.log | tail -4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tconv_gpu.py "tests/test_fp32_gpu.py::test_fp32_resnet18_step_matches_torch_nn" tests/test_graph_k8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for t in 0 1 0 1; do timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 4 8 --updates 256 --tconv $t 2>&1 | grep "ms per" | sed "s/^/tconv=$t /" >> $O/ml.log || exit 1; done
cat $O/ml.log
