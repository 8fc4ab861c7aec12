#!/bin/bash
# default bench line (driver-like) + rocprofv3 kernel stats and fabric counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r4}
timeout -k 10 500 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json | cut -c1-600
bash tools/profile_round.sh $TAG || { echo "PROFILE FAILED"; exit 1; }
echo ok
