# full GPU suite + smoke + default bench (driver-like), logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; exit 1; }
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail gpurun_out/bench_${TAG}.err; exit 1; }
echo ok
