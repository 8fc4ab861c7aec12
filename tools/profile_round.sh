#!/bin/bash
# Run on the GPU box: kernel-trace stats of the bench command plus L2-fabric traffic
# counters in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one pass), for the
# C3 headline unit and for the FITC C4 unit.
# Usage: bash tools/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/...
set -e
TAG=${1:-r2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu --no-grad --no-block"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $BENCH > $OUT/trace.log 2>&1
echo "trace done"
# counters on a shorter run of the headline unit only (every dispatch is serialised and
# sampled), so the per-launch averages match the launches the roofline objects time
PBENCH="bench.py --steps 1 --warmup 0 --no-cpu --no-fitc --no-grad --no-block"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run \
  -- python3 $PBENCH > $OUT/fetch.log 2>&1
echo "fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run \
  -- python3 $PBENCH > $OUT/write.log 2>&1
echo "write done"
python3 tools/traffic.py $OUT > $OUT/traffic_summary.txt
# FITC C4 unit (fit + predict + score) alone
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fitc_fetch -o run \
  -- python3 tools/fitc_unit.py > $OUT/fitc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/fitc_write -o run \
  -- python3 tools/fitc_unit.py > $OUT/fitc_write.log 2>&1
python3 tools/traffic.py $OUT fitc_ > $OUT/fitc_traffic_summary.txt
echo "profile $TAG done"
