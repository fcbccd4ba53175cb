set -o pipefail
# round 5: BERT weight gradients on a side stream (interleaved with the dgrad chain): pair probe + A/B
O=gpurun_out/r5v; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u scripts/gemm_pair_probe.py > $O/pair.log 2>&1 || { tail -5 $O/pair.log; exit 1; }
cat $O/pair.log
MFL_BERT_WGRAD_SIDE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bert_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for t in 0 1 0 1; do
  MFL_BERT_WGRAD_SIDE=$t timeout -k 10 300 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 2>&1 | grep -o '"local_step_ms": [0-9.]*' | sed "s/^/side=$t /" >> $O/bert.log || exit 1
done
cat $O/bert.log
