#!/bin/bash
# persistent factorisation alone (tools/dag_bench): grid sizes, block sizes, one traced launch;
# then the C3 unit's stream-overlap options with the persistent blocks on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3_dagb
O=gpurun_out/r3_dagb
for a in "20 256"; do
  timeout -k 5 60 tools/dag_bench $a >> $O/bench.txt 2>&1 || { echo "DAG_BENCH $a FAILED"; cat $O/bench.txt; exit 1; }
done
timeout -k 5 60 tools/dag_bench 20 256 $O/trace20.csv 5 >> $O/bench.txt 2>&1 || { echo "TRACE FAILED"; exit 1; }
python3 tools/dag_trace.py $O/trace20.csv > $O/trace20.txt 2>&1
cat $O/bench.txt
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --rounds 3 ov=1,dag=1 ov=0,dag=1 ov=1,dag=0 > $O/ab_ov.txt 2>&1 || { echo "AB FAILED"; tail $O/ab_ov.txt; exit 1; }
cat $O/ab_ov.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  --deselect tests/test_gpu_parity.py::test_persistent_factorisation_matches_recursion \
  -k "rccl or profiler or sharing or stats or persistent or shards or surface or asan" > $O/tests_rest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests_rest.log; exit 1; }
tail -3 $O/tests_rest.log
