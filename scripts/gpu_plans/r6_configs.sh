set -o pipefail
# round 6 final tree: BASELINE configs 3 (async, 8 co-located, plain and CKKS PWA),
# 4 (sync + CKKS) and 5 (BERT-base, 1 / 8 co-located learners)
O=gpurun_out/r6/configs; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --secure-aggregation --steps 3 --warmup 1 --exact-updates 0 > $O/config4.log 2>&1 || { tail -5 $O/config4.log; exit 1; }
tail -1 $O/config4.log | cut -c1-300
timeout -k 10 400 python -u benchmarks/async_bench.py > $O/config3.log 2>&1 || { tail -5 $O/config3.log; exit 1; }
tail -1 $O/config3.log | cut -c1-300
timeout -k 10 400 python -u benchmarks/async_bench.py --secure-aggregation > $O/config3_ckks.log 2>&1 || { tail -5 $O/config3_ckks.log; exit 1; }
tail -1 $O/config3_ckks.log | cut -c1-300
for L in 1 8; do
  timeout -k 10 400 python -u benchmarks/bert_bench.py --learners-per-gpu $L --steps 2 --warmup 1 > $O/bert_${L}.log 2>&1 || { tail -5 $O/bert_${L}.log; exit 1; }
  tail -1 $O/bert_${L}.log | cut -c1-400
done
