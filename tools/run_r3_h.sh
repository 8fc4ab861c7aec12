#!/bin/bash
# round 3: FITC (width, side Gram, short-chunk column pass) and the 8-wave GEMM: tests + A/Bs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_h
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_fitc_grad.py -x -v --timeout 300 --timeout-method thread -k "fitc or c4 or c5 or shards or eight_waves or c3_config" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 3 dagwg=0 dagwg=256 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 500 python -u tools/ab_bench.py --config C3 --rounds 3 gw=4,sk=1 gw=8 gw=4,sk=0 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 400 python -u tools/ab_bench.py --config C5 --rounds 2 dagwg=0 dagwg=256 gw=8 > $O/ab_c5.txt 2>&1 || { echo "AB C5 FAILED"; tail -20 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
