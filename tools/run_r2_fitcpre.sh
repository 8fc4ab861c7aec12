#!/bin/bash
# FITC r pre-pass: parity tests, same-box A/B (pre=1: q only, pre=3: q and r), C3/C4 traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_shards.py tests/test_gpu_fitc_grad.py tests/test_gpu_parity.py tests/test_gpu_blockloo.py -k "fitc or c4 or c5 or shard" > gpurun_out/fp_tests.log 2>&1 || { tail -30 gpurun_out/fp_tests.log; exit 1; }
tail -2 gpurun_out/fp_tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 5 pre=1 pre=3 pre=0 > gpurun_out/fp_ab_c4.txt 2>&1 || { cat gpurun_out/fp_ab_c4.txt; exit 1; }
cat gpurun_out/fp_ab_c4.txt
timeout -k 10 300 python -u tools/ab_bench.py --config C5 --rounds 3 pre=1 pre=3 > gpurun_out/fp_ab_c5.txt 2>&1 || { cat gpurun_out/fp_ab_c5.txt; exit 1; }
cat gpurun_out/fp_ab_c5.txt
for c in C3 C4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trp_$c -o run \
    -- python3 tools/trace_unit.py config=$c > gpurun_out/trp_$c.log 2>&1 || exit 1
  python3 tools/fill_profile.py gpurun_out/trp_$c/run_kernel_trace.csv gram_reg 2 > gpurun_out/fill_$c.txt 2>&1
  cat gpurun_out/fill_$c.txt
done
echo ok
