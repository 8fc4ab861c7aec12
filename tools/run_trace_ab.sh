#!/bin/bash
# kernel traces of the production unit under two option sets: bash tools/run_trace_ab.sh "<optsA>" "<optsB>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for o in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr$i -o run \
    -- python3 tools/trace_unit.py $o > gpurun_out/tr$i.log 2>&1 || exit 1
  echo "== $o" >> gpurun_out/trace_ab.txt
  python3 tools/critpath.py gpurun_out/tr$i/run_kernel_trace.csv 2 >> gpurun_out/trace_ab.txt || exit 1
  i=$((i+1))
done
