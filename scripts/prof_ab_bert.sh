#!/bin/bash
# kernel stats of bert_bench under the base and new libraries
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r6s2
so=$(ls metisfl_amd/_ops*.so); cp $so /tmp/new.so
for v in base new; do
  if [ $v = base ]; then cp build/ab/_ops_base.so $so; else cp /tmp/new.so $so; fi
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6s2/p_$v -o run -- python3 $R/benchmarks/bert_bench.py --steps 1 --warmup 1 --local-steps 10 > $R/gpurun_out/r6s2/p_$v.log 2>&1) || { cp /tmp/new.so $so; exit 1; }
  f=$(find gpurun_out/r6s2/p_$v -name "*kernel_stats.csv" | head -1)
  python scripts/kstats.py $f 20 12 > gpurun_out/r6s2/kstats_$v.txt
  rm -rf gpurun_out/r6s2/p_$v
done
cp /tmp/new.so $so
