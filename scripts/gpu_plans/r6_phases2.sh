set -o pipefail
mkdir -p gpurun_out/r6/phases2
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exact-updates 0 > gpurun_out/r6/phases2/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null &&
PYTHONPATH=. timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/phases2/prof -o step -- python3 scripts/multi_learner_probe.py --groups 8 --updates 64 > gpurun_out/r6/phases2/prof.log 2>&1
