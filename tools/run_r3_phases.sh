#!/bin/bash
# round 3: bench with the per-phase record (fit / predict / score), short run
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_phases
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "predict or score or c3_config or fitc" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-grad --no-block > $O/bench.json 2> $O/bench.log || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('C3', d['ms_per_step'], d['phases'])
for k,v in d['fitc'].items(): print(k, v['ms_per_step'], v['phases'])"
