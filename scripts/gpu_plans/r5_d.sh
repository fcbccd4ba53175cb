set -o pipefail
# round 5: 128-pixel dgrad tile in the backward pair (MFL_C32_PAIR_DBM): numerics, one learner, 8 co-located
O=gpurun_out/r5d; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
MFL_C32_PAIR_DBM=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp32_gpu.py tests/test_graph_k8_gpu.py -k "pair or oracle or k8 or colocated_streams" > $O/t128.log 2>&1 || { tail -40 $O/t128.log; exit 1; }
tail -2 $O/t128.log
for d in 64 128 64 128; do MFL_C32_PAIR_DBM=$d timeout -k 10 300 python -u scripts/step_prof.py --steps 300 --warmup 40 2>&1 | grep "ms per" | sed "s/^/dbm=$d /" >> $O/one.log || exit 1; done
cat $O/one.log
for d in 64 128 64 128; do MFL_C32_PAIR_DBM=$d timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "ms per" | sed "s/^/dbm=$d /" >> $O/ml.log || exit 1; done
cat $O/ml.log
