#!/bin/bash
# Round 6: GPS_OPT_FITC_DEP — its GPU tests, a same-box C4 A/B (and factorisation widths), and one
# C4 unit's kernel timeline with the dependent row norms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fitc_dep.py tests/test_gpu_shards.py::test_local_group_late_joiner tests/test_gpu_shards.py::test_local_group_reinit_and_duplicate_rank -m gpu \
  > gpurun_out/r6a_dep_tests.log 2>&1 || { tail -30 gpurun_out/r6a_dep_tests.log; exit 1; }
tail -3 gpurun_out/r6a_dep_tests.log
timeout -k 10 400 python -u tools/ab_bench.py --config C4 --steps 10 --rounds 5 dep=0 dep=1 dep=1,dagwg=96 dep=1,dagwg=64 dep=1,dagwg=160 \
  > gpurun_out/r6a_dep_ab_c4.txt 2>&1 || exit 1
cat gpurun_out/r6a_dep_ab_c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6a_c4tl -o c4tl \
  -- python3 tools/fitc_unit.py > gpurun_out/r6a_c4tl.log 2>&1 || exit 1
python3 tools/fitc_timeline.py $(ls gpurun_out/r6a_c4tl/*/*kernel_trace.csv gpurun_out/r6a_c4tl/*kernel_trace.csv 2>/dev/null | head -1) 1 > gpurun_out/r6a_c4_timeline.txt
tail -45 gpurun_out/r6a_c4_timeline.txt
