#!/bin/bash
# Round 6: same-box C4 A/B of GPS_OPT_FITC_DEP (0 off, 1 q behind Lm, 2 q and r) and factorisation
# widths, then one C4 unit's kernel timeline at the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6b}
timeout -k 10 400 python -u tools/ab_bench.py --config C4 --steps 10 --rounds 5 ${VARIANTS:-dep=0 dep=1 dep=2 dep=1,dagwg=96 dep=1,dagwg=64} \
  > gpurun_out/${T}_dep_ab_c4.txt 2>&1 || exit 1
cat gpurun_out/${T}_dep_ab_c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_c4tl -o c4tl \
  -- python3 tools/fitc_unit.py > gpurun_out/${T}_c4tl.log 2>&1 || exit 1
