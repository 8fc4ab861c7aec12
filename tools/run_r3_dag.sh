#!/bin/bash
# round 3: first GPU run of the persistent factorisation — its tests, then a same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "persistent or potrf or c3_config_vs or golden" > gpurun_out/r3_dag_tests.log 2>&1 || { echo "DAG TESTS FAILED"; tail -30 gpurun_out/r3_dag_tests.log; exit 1; }
tail -3 gpurun_out/r3_dag_tests.log
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --rounds 3 dag=0 dag=1,dagt=20 dag=1,dagt=10 dag=1,dagt=40 > gpurun_out/r3_dag_ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 gpurun_out/r3_dag_ab_c3.txt; exit 1; }
cat gpurun_out/r3_dag_ab_c3.txt
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 3 dag=0 dag=1,dagt=20 dag=1,dagt=16 > gpurun_out/r3_dag_ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 gpurun_out/r3_dag_ab_c4.txt; exit 1; }
cat gpurun_out/r3_dag_ab_c4.txt
