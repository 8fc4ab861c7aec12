set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG:-r1f}.json 2> gpurun_out/bench_${TAG:-r1f}.err || { echo "BENCH FAILED"; exit 1; }
echo ok
