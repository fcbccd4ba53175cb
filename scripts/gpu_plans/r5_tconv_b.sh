set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/tconv_step_diff.py > $O/diff.log 2>&1; cat $O/diff.log | grep -v amdgpu.ids
