set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sharing or golden" > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 bash tools/run_gemm_bench.sh rowsq > gpurun_out/rowsq_map5.txt 2>&1 || exit 1
cat gpurun_out/rowsq_map5.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r2c.json 2> gpurun_out/bench_r2c.err || exit 1
echo ok
