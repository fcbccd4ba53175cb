set -o pipefail
# round 5: fused optimizer grid cap A/B (BERT AdamW over 110M parameters; the ResNet step's end-of-step launch)
O=gpurun_out/r5o; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for c in 2048 8192 2048 8192; do
  MFL_OPT_GRID_CAP=$c timeout -k 10 300 python -u benchmarks/bert_bench.py --steps 2 --warmup 1 2>&1 | grep -o '"local_step_ms": [0-9.]*' | sed "s/^/cap=$c bert /" >> $O/ab.log || exit 1
  MFL_OPT_GRID_CAP=$c timeout -k 10 200 python -u scripts/step_prof.py --steps 800 2>&1 | grep "local update" | sed "s/^/cap=$c one: /" >> $O/ab.log || exit 1
done
cat $O/ab.log
