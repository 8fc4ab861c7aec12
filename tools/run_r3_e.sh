#!/bin/bash
# round 3: GPU suite at the LOO-finaliser build, then the fork range with the stream-K tail on
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_e
mkdir -p $O
TAG=r3e bash tools/run_r3_suite.sh || exit 1
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --rounds 3 forkmax=0 forkmax=77 ov=0 > $O/ab_c3_fork.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3_fork.txt; exit 1; }
cat $O/ab_c3_fork.txt
