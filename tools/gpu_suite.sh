#!/bin/bash
# full GPU suite (parity floors recorded) + smoke; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r4}
export GPS_PARITY_FLOORS=$PWD/gpurun_out/parity_floors_${TAG}.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_suite_${TAG}.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" gpurun_out/gpu_suite_${TAG}.log | head -30; tail -30 gpurun_out/gpu_suite_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_suite_${TAG}.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
echo ok
