set -o pipefail
# round 5: 8-learner co-located kernel stats; exact-products regression: round-4 start tree vs this tree, same box
O=gpurun_out/r5f; mkdir -p $O
export TMPDIR=/tmp
R=$PWD
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/multi_learner_probe.py --groups 8 --updates 128 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 1 45 > $O/kstats8.txt && head -50 $O/kstats8.txt
for t in old new old new; do
  if [ $t = old ]; then D=$R/build/wt_adbe; else D=$R; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 > $R/$O/bench_$t.log 2>&1) || { tail -20 $R/$O/bench_$t.log; exit 1; }
  tail -1 $R/$O/bench_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['round_ms'],1), round(d['train_ms_mean'],1), round(d['conv_products_exact']['ms_per_update'],3))"
done
