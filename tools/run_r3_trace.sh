#!/bin/bash
# kernel trace of the C3 production unit (DAG on / off) + critical-path summaries; bench without CPU legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3_trace
mkdir -p $OUT
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/dag$v -o run -- python3 tools/trace_unit.py dag=$v > $OUT/dag$v.log 2>&1 || { echo "TRACE $v FAILED"; exit 1; }
  f=$(ls $OUT/dag$v/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/dag$v/run_kernel_trace.csv)
  python3 tools/critpath.py $f 1 > $OUT/critpath_dag$v.txt 2>&1
done
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-grad --no-block > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail $OUT/bench.err; exit 1; }
echo ok
