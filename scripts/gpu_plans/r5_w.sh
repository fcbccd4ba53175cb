set -o pipefail
# round 5: where a test-set evaluation's time goes (fp32 ResNet-18, 10k samples, BN inference)
O=gpurun_out/r5w; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_probe.py --batches 256,512 --reps 3 > $O/eval.log 2>&1 || { tail -5 $O/eval.log; exit 1; }
cat $O/eval.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/eval_probe.py --batches 256 --reps 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cut -d, -f1-5 $(find $O/prof -name "*kernel_stats.csv") | head -30
