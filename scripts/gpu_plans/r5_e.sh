set -o pipefail
# round 5: config 3 on the unified async core (8 co-located learners), plain and CKKS PWA
O=gpurun_out/r5e; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/async_bench.py --gpus 1 --learners 8 --tasks 3 > $O/async8.log 2>&1 || { tail -20 $O/async8.log; exit 1; }
tail -1 $O/async8.log | cut -c1-300
timeout -k 10 600 python -u benchmarks/async_bench.py --gpus 1 --learners 8 --tasks 3 --secure-aggregation > $O/async8_ckks.log 2>&1 || { tail -20 $O/async8_ckks.log; exit 1; }
tail -1 $O/async8_ckks.log | cut -c1-300
