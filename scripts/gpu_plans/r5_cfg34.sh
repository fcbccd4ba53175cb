set -o pipefail
# round 5 final: BASELINE configs 3 (async, 8 co-located, plain and CKKS PWA) and 4 (sync + CKKS) on the final tree
O=gpurun_out/r5c34; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --secure-aggregation --steps 2 --warmup 1 > $O/config4.log 2>&1 || { tail -5 $O/config4.log; exit 1; }
tail -1 $O/config4.log | cut -c1-300
timeout -k 10 400 python -u benchmarks/async_bench.py > $O/config3.log 2>&1 || { tail -5 $O/config3.log; exit 1; }
tail -1 $O/config3.log | cut -c1-300
timeout -k 10 400 python -u benchmarks/async_bench.py --secure-aggregation > $O/config3_ckks.log 2>&1 || { tail -5 $O/config3_ckks.log; exit 1; }
tail -1 $O/config3_ckks.log | cut -c1-300
