set -o pipefail
# round 5: pair ring 2 vs 3 with 2 co-located learners (the N = 4 point of the bench)
O=gpurun_out/r5i; mkdir -p $O
export PYTHONPATH=$PWD
for r in 3 2 3 2; do timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 2 --updates 384 --pair-ring $r 2>&1 | grep "ms per" | sed "s/^/ring=$r /" >> $O/g2.log || exit 1; done
cat $O/g2.log
