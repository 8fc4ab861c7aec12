#!/bin/bash
# Same-box A/B on the GPU: the C3 headline (and the FITC C4 unit) with ab/libgpscore_<base>.so
# (tools/build_ref_lib.sh; moved to tbin/, which travels with gpurun, or $LIBDIR) against the
# working library, interleaved, 2 rounds.
#   bash tools/ab_lib.sh base   -> gpurun_out/ab_<base>_{ref,cur}_<r>.json
set -o pipefail
cd $GRAFT_REPO_ROOT
NAME=${1:-base}
B="bench.py --steps 5 --warmup 2 --no-grad --no-block --no-cpu"
for r in 1 2; do
  GPSCORE_LIB=$PWD/${LIBDIR:-tbin}/libgpscore_$NAME.so timeout -k 5 200 python -u $B > gpurun_out/ab_${NAME}_ref_$r.json 2>/dev/null || exit 1
  timeout -k 5 200 python -u $B > gpurun_out/ab_${NAME}_cur_$r.json 2>/dev/null || exit 1
done
python3 - <<PY
import json
for r in (1, 2):
    for v in ("ref", "cur"):
        d = json.load(open(f"gpurun_out/ab_${NAME}_{v}_{r}.json"))
        print(r, v, "C3 %.2f ms" % d["ms_per_step"], "C4 %.3f ms" % d["fitc"]["C4"]["ms_per_step"],
              "C5 %.2f ms" % d["fitc"]["C5"]["ms_per_step"])
PY
