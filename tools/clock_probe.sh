#!/bin/bash
# Effective shader clock per kernel under load (MI355X_MICROARCH.md 'DVFS give-back':
# GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time) and MFMA-pipe busy cycles, one C3 unit,
# counters in their own pass.
set -e
OUT=gpurun_out/clock
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace \
  --output-format csv -d $OUT/pmc -o run \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-fitc --no-grad --no-block > $OUT/pmc.log 2>&1
python3 tools/clock_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
