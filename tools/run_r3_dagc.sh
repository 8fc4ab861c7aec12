#!/bin/bash
# persistent factorisation alone: load-group depth x queue order, then traces
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_dagc
mkdir -p $O
for go in "2 0" "2 1" "3 0" "3 1" "4 1"; do
  timeout -k 5 60 tools/dag_bench 20 256 - 20 $go >> $O/bench.txt 2>&1 || { echo "DAG_BENCH $go FAILED"; cat $O/bench.txt; exit 1; }
done
for go in "3 1" "3 0"; do
  set -- $go
  timeout -k 5 60 tools/dag_bench 20 256 $O/trace_g$1_o$2.csv 3 $go >> $O/bench.txt 2>&1 || { echo "TRACE FAILED"; exit 1; }
  python3 tools/dag_trace.py $O/trace_g$1_o$2.csv > $O/trace_g$1_o$2.txt 2>&1
done
for go in "3 1" "3 0"; do
  timeout -k 5 60 tools/dag_bench 40 256 - 10 $go >> $O/bench.txt 2>&1 || { echo "DAG_BENCH 40 FAILED"; exit 1; }
  timeout -k 5 60 tools/dag_bench 10 256 - 10 $go >> $O/bench.txt 2>&1 || { echo "DAG_BENCH 10 FAILED"; exit 1; }
done
cat $O/bench.txt
