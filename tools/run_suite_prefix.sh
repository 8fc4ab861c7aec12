#!/bin/bash
# The GPU suite's own collection (torch imported by test_host_logic, so torch's bundled HIP
# runtime serves libgpscore.so) up to the FITC gradient module: the order that exposed the
# graph-exec destroy crash (api.hip potrf_inv, kMaxGraphs); then the same modules alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --ignore=tests/test_gpu_parity.py --ignore=tests/test_gpu_shards.py --ignore=tests/test_gpu_surface.py --ignore=tests/test_gpu_grad.py > gpurun_out/prefix_full.log 2>&1
echo "collection-order rc=$?"; grep -c PASSED gpurun_out/prefix_full.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_asan.py tests/test_gpu_blockloo.py tests/test_gpu_experiment.py tests/test_gpu_fitc_grad.py > gpurun_out/prefix_sub.log 2>&1
echo "modules-alone rc=$?"; tail -1 gpurun_out/prefix_sub.log
