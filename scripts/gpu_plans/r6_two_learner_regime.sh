# A/B: the co-located kernel regime (2-stage pair ring, co-located plans,
# halo conv off at 4x4) for TWO learners per GPU (the bench's N = 4 point)
set -o pipefail
mkdir -p gpurun_out/r6/reg2
for rep in 1 2 3; do
  echo "=== rep $rep default" >> gpurun_out/r6/reg2/ab.log
  PYTHONPATH=. timeout -k 10 200 python scripts/multi_learner_probe.py --groups 2 --updates 384 >> gpurun_out/r6/reg2/ab.log 2>&1 || exit 1
  echo "=== rep $rep regime" >> gpurun_out/r6/reg2/ab.log
  MFL_COLOC_PAIR_RING_MIN=2 PYTHONPATH=. timeout -k 10 200 python scripts/multi_learner_probe.py --groups 2 --updates 384 >> gpurun_out/r6/reg2/ab.log 2>&1 || exit 1
done
