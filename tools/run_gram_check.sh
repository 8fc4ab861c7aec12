set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "gram or golden or shapes or c3 or c2" > gpurun_out/gramchk.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-grad --no-block > gpurun_out/bench_gchk_$r.json 2>/dev/null || { echo "BENCH FAILED"; exit 1; }
done
echo ok
