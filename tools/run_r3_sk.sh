#!/bin/bash
# round 3: stream-K tail — its tests and the sharded block-LOO tests, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_sk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -v --timeout 200 --timeout-method thread \
  -k "stream_k or persistent or c3_config or large_properties or blockloo or shards" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --rounds 4 sk=0 sk=1 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
true

