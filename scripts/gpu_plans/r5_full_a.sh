set -o pipefail
# round 5: whole GPU suite after the async-core rewrite, smoke, a 1-GPU bench
O=gpurun_out/r5full; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -2 $O/bench.log
