#!/bin/bash
# A library change against a base build (tools/build_ref_lib.sh + tbin/dag_bench_base): the persistent
# 2560-block time (dag_bench, interleaved) and the FITC block-LOO gradient floor with each library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6d}
for r in 1 2 3; do
  timeout -k 10 120 tbin/dag_bench_base 20 256 - 30 > gpurun_out/${T}_dag_base_$r.txt 2>&1 || exit 1
  timeout -k 10 120 tbin/dag_bench 20 256 - 30 > gpurun_out/${T}_dag_new_$r.txt 2>&1 || exit 1
done
grep -h -i "ms\|err" gpurun_out/${T}_dag_base_*.txt | head -12
echo ---
grep -h -i "ms\|err" gpurun_out/${T}_dag_new_*.txt | head -12
GPSCORE_LIB=$PWD/tbin/libgpscore_base.so timeout -k 10 300 python -u tools/fitc_noise_localise.py gpurun_out/${T}_noise_base.json > gpurun_out/${T}_noise_base.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/fitc_noise_localise.py gpurun_out/${T}_noise_new.json > gpurun_out/${T}_noise_new.log 2>&1 || exit 1
python3 - <<PY
import json
for v in ("base", "new"):
    r = json.load(open("gpurun_out/${T}_noise_%s.json" % v))
    print(v, "gpu floor", [round(f["grad"], 12) for f in r["gpu_floor"]], "oracle floor",
          [round(f["grad"], 12) for f in r["oracle_floor"]], "Lb_inv diff", r["intermediate_diff"]["Lb_inv"],
          "gpu_vs_oracle", r["gpu_vs_oracle"])
PY
