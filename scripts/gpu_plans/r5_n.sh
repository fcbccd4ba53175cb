set -o pipefail
# round 5: conv32 epilogue reads issued up front: fp32 numerics, one learner, 8 co-located; LN block sweep
O=gpurun_out/r5n; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_graph_k8_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do timeout -k 10 300 python -u scripts/step_prof.py --steps 300 --warmup 40 2>&1 | grep "ms per" >> $O/one.log || exit 1; done
cat $O/one.log
for i in 1 2; do timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "ms per" >> $O/ml.log || exit 1; done
cat $O/ml.log
for b in 128 256 512 1024; do MFL_LN_BWD_BLOCKS=$b timeout -k 10 120 python scripts/ln_micro.py || exit 1; done
