set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG:-r1e}.json 2> gpurun_out/bench_${TAG:-r1e}.err || { echo "BENCH FAILED"; exit 1; }
echo ok
