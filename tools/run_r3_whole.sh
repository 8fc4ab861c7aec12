#!/bin/bash
# round 3: whole-tile tasks in the persistent factorisation — standalone bench (strips vs whole,
# T = 20 / 32 / 40), a traced launch, the DAG tests, then same-box C3 / C4 A/Bs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_whole
mkdir -p $O
for a in "20 256 - 20 3 1 0" "20 256 - 20 3 1 1" "16 256 - 20 3 1 0" "16 256 - 20 3 1 1" "40 256 - 10 3 1 0" "40 256 - 10 3 1 1"; do
  echo "whole=${a: -1}: $(timeout -k 5 60 tools/dag_bench $a 2>&1 | tail -1)" >> $O/bench.txt || { echo "DAG_BENCH $a FAILED"; cat $O/bench.txt; exit 1; }
done
timeout -k 5 60 tools/dag_bench 40 256 $O/trace40.csv 3 3 1 1 >> $O/bench.txt 2>&1 || { echo "TRACE FAILED"; exit 1; }
python3 tools/dag_trace.py $O/trace40.csv > $O/trace40.txt 2>&1
cat $O/bench.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "persistent" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --rounds 3 dagw=0,dagt=20 dagw=1,dagt=20 dagw=1,dagt=40 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 200 python -u tools/ab_bench.py --config C4 --rounds 3 dagw=0 dagw=1 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
