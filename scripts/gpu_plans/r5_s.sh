set -o pipefail
# round 5: same-box bench A/B, tree before the conv output-stage change (13eae40) vs this tree
O=gpurun_out/r5s; mkdir -p $O
R=$PWD
for t in old new old new; do
  if [ $t = old ]; then D=$R/build/wt_head; else D=$R; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 --exact-updates 0 > $R/$O/bench_$t.log 2>&1) || { tail -20 $R/$O/bench_$t.log; exit 1; }
  tail -1 $R/$O/bench_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['round_ms'],1), round(d['train_ms_mean'],1), round(d['community_eval_ms_mean'],1))" | tee -a $R/$O/ab.log
done
