#!/bin/bash
# round 3: cohort order of the predictive TRMM — its tests, a same-box C3 A/B, then kernel
# trace and L2-fabric counters of both orders in one process (different kernel names)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_coh
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "cohort or c3_config" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --rounds 4 coh=0 coh=1 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
  -- python3 tools/ab_bench.py --config C3 --rounds 1 --steps 2 coh=0 coh=1 > $O/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $O/trace.log; exit 1; }
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run \
  -- python3 tools/ab_bench.py --config C3 --rounds 1 --steps 1 coh=0 coh=1 > $O/fetch.log 2>&1 || { echo "FETCH FAILED"; tail -20 $O/fetch.log; exit 1; }
echo "fetch done"
true
