# Run selected GPU tests on the box: bash tools/run_gpu_tests.sh <log-tag> <pytest args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/tests_$TAG.log
exit $rc
