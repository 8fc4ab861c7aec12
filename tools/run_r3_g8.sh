#!/bin/bash
# round 3: one-shot strip loads (group 8) vs 3-chunk groups — standalone DAG bench, then
# same-box end-to-end A/B on C3 and C4, then the default bench line + rocprofv3 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_g8
mkdir -p $O
for go in "3 1" "8 1" "3 1" "8 1"; do
  timeout -k 5 60 tools/dag_bench 20 256 - 20 $go >> $O/bench.txt 2>&1 || { echo "DAG_BENCH $go FAILED"; cat $O/bench.txt; exit 1; }
done
timeout -k 5 60 tools/dag_bench 16 256 - 20 3 1 >> $O/bench.txt 2>&1 && timeout -k 5 60 tools/dag_bench 16 256 - 20 8 1 >> $O/bench.txt 2>&1 || { echo "DAG_BENCH 16 FAILED"; exit 1; }
timeout -k 5 60 tools/dag_bench 20 256 $O/trace_g8.csv 3 8 1 >> $O/bench.txt 2>&1 || { echo "TRACE FAILED"; exit 1; }
python3 tools/dag_trace.py $O/trace_g8.csv > $O/trace_g8.txt 2>&1
cat $O/bench.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "persistent" > $O/tests.log 2>&1 || { echo "DAG TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --rounds 3 dagg=3 dagg=8 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 200 python -u tools/ab_bench.py --config C4 --rounds 3 dagg=3 dagg=8 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
TAG=r3a bash tools/run_r3_bench_prof.sh
