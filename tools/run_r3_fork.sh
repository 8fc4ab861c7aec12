#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_fork
mkdir -p $O
timeout -k 10 500 python -u tools/ab_bench.py --config C3 --rounds 3 dag=0,fork=1 dag=1,fork=1 dag=1,fork=39 dag=1,fork=78 > $O/ab_c3.txt 2>&1 || { echo "AB FAILED"; tail $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 3 dag=0 dag=1 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
