#!/bin/bash
# Run on the GPU box: kernel-trace stats of the bench command plus HBM traffic
# counters in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one pass).
# Usage: bash tools/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/...
set -e
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $BENCH > $OUT/trace.log 2>&1
# counters on a shorter run of the headline unit only (every dispatch is serialised and
# sampled), so the per-launch averages match the launches the roofline objects time
PBENCH="bench.py --steps 1 --warmup 0 --no-cpu --no-fitc --no-grad --no-block"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run \
  -- python3 $PBENCH > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run \
  -- python3 $PBENCH > $OUT/write.log 2>&1
python3 tools/traffic.py $OUT > $OUT/traffic_summary.txt
echo "profile $TAG done"
