#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_fork2
mkdir -p $O
timeout -k 10 500 python -X faulthandler -u tools/ab_bench.py --config C3 --rounds 3 forkmax=0 forkmax=77 forkmax=38 > $O/ab_c3.txt 2>&1 || { echo "AB FAILED"; tail $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
