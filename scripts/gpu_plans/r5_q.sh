set -o pipefail
# round 5: pipelined optimizer loops (tails + fused launch): numerics + same-box A/B (old = HEAD worktree)
O=gpurun_out/r5q; mkdir -p $O
R=$PWD
export PYTHONPATH=$R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "opt or fp32 or resnet or bert or k8" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for t in old new old new; do
  if [ $t = old ]; then D=$R/build/wt_head; else D=$R; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep "ms per" | sed "s/^/$t /") >> $O/ml.log || exit 1
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u scripts/step_prof.py --steps 300 --warmup 40 2>&1 | grep "ms per" | sed "s/^/$t /") >> $O/one.log || exit 1
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 2>&1 | grep -o '"local_step_ms": [0-9.]*' | sed "s/^/$t /") >> $O/bert.log || exit 1
done
cat $O/ml.log $O/one.log $O/bert.log
