#!/bin/bash
# Kernel-trace only (no counters): per-kernel durations and the idle gaps between
# consecutive dispatches of one C3 unit, to size launch overhead on the dependent chain.
set -e
OUT=gpurun_out/gaps
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-fitc > $OUT/trace.log 2>&1
python3 tools/gap_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
