#!/bin/bash
# Same-box C4 A/B of GPS_OPT_FITC_DEP (0 off, 1 on) and factorisation
# widths (VARIANTS), then one C4 unit's kernel timeline at the default (TAG names the outputs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6b}
timeout -k 10 400 python -u tools/ab_bench.py --config C4 --steps 10 --rounds 5 ${VARIANTS:-dep=0 dep=1} \
  > gpurun_out/${T}_dep_ab_c4.txt 2>&1 || exit 1
cat gpurun_out/${T}_dep_ab_c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_c4tl -o c4tl \
  -- python3 tools/fitc_unit.py > gpurun_out/${T}_c4tl.log 2>&1 || exit 1
