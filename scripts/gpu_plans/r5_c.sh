set -o pipefail
# round 5: device async PWA test; same-box pair-ring A/B (bf16x3 and exact); 8-learner co-located kernel stats
O=gpurun_out/r5c2; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_colocated_gpu.py > $O/coloc.log 2>&1 || { tail -40 $O/coloc.log; exit 1; }
tail -3 $O/coloc.log
for r in 3 2 3 2; do timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 --pair-ring $r 2>&1 | grep "ms per" | sed "s/^/ring=$r /" >> $O/ring.log || exit 1; done
cat $O/ring.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/multi_learner_probe.py --groups 8 --updates 128 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv") 1 40 > $O/kstats8.txt && head -45 $O/kstats8.txt
timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 128 --conv-products exact 2>&1 | grep "ms per" | sed "s/^/exact /" >> $O/exact.log || exit 1
cat $O/exact.log
for k in MFL_OPT_TAIL=0 MFL_C32_WSTORE=0 MFL_BN_PREMASK=0 MFL_BN_BWD_PAIR=0 MFL_INPLACE_RESGRAD=0 NONE=1; do env $k timeout -k 10 300 python -u scripts/multi_learner_probe.py --groups 8 --updates 128 --conv-products exact 2>&1 | grep "ms per" | sed "s/^/exact $k /" >> $O/exact.log || exit 1; done
cat $O/exact.log
