#!/bin/bash
# the default bench line alone (driver-like): gpurun_out/bench_<TAG>.json
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r4}
timeout -k 10 ${TMO:-500} python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail gpurun_out/bench_${TAG}.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_${TAG}.json 2>/dev/null || cut -c1-600 gpurun_out/bench_${TAG}.json
