set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fitc_grad.py tests/test_gpu_blockloo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fitcgrad.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/bench_fg.json 2> gpurun_out/bench_fg.err || { echo "BENCH FAILED"; exit 1; }
echo ok
