set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_all.log; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/bench_${TAG:-r2a}.json 2> gpurun_out/bench_${TAG:-r2a}.err || { echo "BENCH FAILED"; exit 1; }
echo ok
