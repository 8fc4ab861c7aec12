#!/bin/bash
# round 3: full GPU suite, then C4 timing and the stream-K mechanism check (overlap off)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_c
mkdir -p $O
TAG=r3c bash tools/run_r3_suite.sh || exit 1
timeout -k 10 200 python -u tools/ab_bench.py --config C4 --rounds 3 sk=1 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --rounds 3 ov=0,sk=0 ov=0,sk=1 sk=1,sprio=0 sk=1,sprio=1 > $O/ab_c3_ov.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3_ov.txt; exit 1; }
cat $O/ab_c3_ov.txt
