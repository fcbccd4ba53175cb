set -o pipefail
# round 5: GEMM output stage reads one chunk ahead: numerics + same-box A/B + kernel time
O=gpurun_out/r5u; mkdir -p $O
R=$PWD
export PYTHONPATH=$R TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bert_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for t in old new old new; do
  if [ $t = old ]; then D=$R/build/wt_head; else D=$R; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 2>&1 | grep -o '"local_step_ms": [0-9.]*' | sed "s/^/$t /") >> $O/bert.log || exit 1
done
cat $O/bert.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bert_bench.py --steps 1 --warmup 0 --local-steps 10 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -h "gemm_pp" $(find $O/prof -name "*kernel_stats.csv") | cut -c1-200
