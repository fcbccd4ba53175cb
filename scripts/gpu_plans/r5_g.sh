set -o pipefail
# round 5: co-located step kernel time, paired backward vs throughput (tconv) backward
O=gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for t in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t$t -o run -- python3 scripts/multi_learner_probe.py --groups 8 --updates 128 --tconv $t > $O/prof_t$t.log 2>&1 || { tail -20 $O/prof_t$t.log; exit 1; }
  grep "ms per" $O/prof_t$t.log
  python3 scripts/kstats.py $(find $O/prof_t$t -name "*kernel_stats.csv" | head -1) 1 30 > $O/kstats_t$t.txt && tail -1 $O/kstats_t$t.txt
done
head -14 $O/kstats_t1.txt
