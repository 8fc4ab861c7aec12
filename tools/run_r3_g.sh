#!/bin/bash
# round 3: FITC after the width / column-pass changes — FITC tests, C4 and C5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_fitc_grad.py -x -v --timeout 300 --timeout-method thread -k "fitc or c4 or c5 or shards" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 3 dagwg=0 dagwg=256 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 400 python -u tools/ab_bench.py --config C5 --rounds 2 dagwg=0 dagwg=256 > $O/ab_c5.txt 2>&1 || { echo "AB C5 FAILED"; tail -20 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
