#!/bin/bash
# same-box A/B of two library builds: bash tools/run_lib_ab.sh <lib-A.so> <lib-B.so> <config> <rounds>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 ${4:-3}); do
  for L in "$1" "$2"; do
    GPSCORE_LIB=$PWD/$L timeout -k 10 300 python -u tools/ab_bench.py --config $3 --rounds 1 map=0 2>&1 | sed "s|^|$(basename $L) |"
  done
done
