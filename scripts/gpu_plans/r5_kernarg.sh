set -o pipefail
# round 5: HIP runtime knob A/B -- kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) for the
# graph-replayed step: one learner (latency-bound) and 8 co-located learners
O=gpurun_out/r5k; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for k in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python -u scripts/step_prof.py --steps 800 2>&1 | grep -v amdgpu.ids | sed "s/^/kernarg=$k one: /" >> $O/ab.log || exit 1
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python -u scripts/multi_learner_probe.py --groups 8 --updates 256 2>&1 | grep -v amdgpu.ids | tail -2 | sed "s/^/kernarg=$k eight: /" >> $O/ab.log || exit 1
done
cat $O/ab.log
