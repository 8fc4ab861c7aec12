set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_gram.json 2> gpurun_out/bench_gram.err || { echo "BENCH FAILED"; exit 1; }
echo ok
