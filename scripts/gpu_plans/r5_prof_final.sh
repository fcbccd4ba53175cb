set -o pipefail
# round 5 final: rocprofv3 kernel statistics of the final tree's one-learner step and of the BERT step
O=gpurun_out/r5pf; mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 scripts/step_prof.py --steps 150 > $O/step.log 2>&1 || { tail -5 $O/step.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bert -o run -- python3 benchmarks/bert_bench.py --steps 1 --warmup 0 --local-steps 10 > $O/bert.log 2>&1 || { tail -5 $O/bert.log; exit 1; }
ls $O/step $O/bert
