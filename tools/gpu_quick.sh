#!/bin/bash
# a subset of the GPU suite (PYTEST_K) with its own log; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-q}
export GPS_PARITY_FLOORS=$PWD/gpurun_out/parity_floors_${TAG}.json
timeout -k 10 ${TMO:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/quick_${TAG}.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" gpurun_out/quick_${TAG}.log | head -30; tail -40 gpurun_out/quick_${TAG}.log; exit 1; }
tail -3 gpurun_out/quick_${TAG}.log
