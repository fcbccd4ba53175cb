set -o pipefail
# round 5 final: BASELINE config 5 as 1 / 4 / 8 co-located BERT-base learners on one GPU (final tree)
O=gpurun_out/r5b8; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for L in 1 4 8; do
  timeout -k 10 400 python -u benchmarks/bert_bench.py --learners-per-gpu $L --steps 2 --warmup 1 > $O/bert_${L}.log 2>&1 || { tail -5 $O/bert_${L}.log; exit 1; }
  tail -1 $O/bert_${L}.log | cut -c1-400
done
