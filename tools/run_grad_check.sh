set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_blockloo.py tests/test_gpu_experiment.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gradchk.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu --no-fitc --no-block > gpurun_out/bench_gradchk.json 2>/dev/null || { echo "BENCH FAILED"; exit 1; }
echo ok
