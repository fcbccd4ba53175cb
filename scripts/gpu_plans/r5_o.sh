set -o pipefail
# round 5: same-box A/B of the conv32 epilogue prefetch (old = committed HEAD worktree, new = this tree)
O=gpurun_out/r5o; mkdir -p $O
R=$PWD
for t in old new old new; do
  if [ $t = old ]; then D=$R/build/wt_head; else D=$R; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "ms per" | sed "s/^/$t /") >> $O/ml.log || exit 1
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u scripts/step_prof.py --steps 300 --warmup 40 2>&1 | grep "ms per" | sed "s/^/$t /") >> $O/one.log || exit 1
done
cat $O/ml.log $O/one.log
