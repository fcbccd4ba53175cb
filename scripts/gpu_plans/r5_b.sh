set -o pipefail
# round 5: 8-stream co-location pins, exact-mode pair-ring A/B, BERT config 5 with 4 / 8 learners
O=gpurun_out/r5b; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_graph_k8_gpu.py > $O/k8.log 2>&1 || { tail -40 $O/k8.log; exit 1; }
grep -E "rel|passed|failed" $O/k8.log | tail -20
MFL_COLOC_PAIR_RING=0 timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > $O/bench_ring0.log 2>&1 || { tail -20 $O/bench_ring0.log; exit 1; }
tail -1 $O/bench_ring0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ring0', d['ms_per_step'], d['conv_products_exact']['ms_per_update'])"
timeout -k 10 900 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 --learners-per-gpu 4 > $O/bert4.log 2>&1 || { tail -30 $O/bert4.log; exit 1; }
tail -2 $O/bert4.log
timeout -k 10 900 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 --learners-per-gpu 8 > $O/bert8.log 2>&1 || { tail -30 $O/bert8.log; exit 1; }
tail -2 $O/bert8.log
