#!/bin/bash
# Same-box A/B of the whole bench between a reference tree (tbin/<ref>/: bench.py + the package with
# its own libgpscore.so, e.g. the previous round's final commit built with its own binding) and the
# working tree, interleaved: C3 / C4 / C5 ms per step and C3 production vs kernel-accounting time.
#   REF=r5 ROUNDS=3 bash tools/tree_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
REF=${REF:-r5}; T=${TAG:-tree_ab}
B="--steps ${STEPS:-5} --warmup 2 --no-grad --no-block --no-cpu"
for r in $(seq 1 ${ROUNDS:-3}); do
  (cd tbin/$REF && timeout -k 10 300 python -u bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/${T}_ref_$r.json 2>/dev/null) || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_cur_$r.json 2>/dev/null || exit 1
done
python3 - <<PY
import json
for r in range(1, ${ROUNDS:-3} + 1):
    for v in ("ref", "cur"):
        d = json.load(open(f"gpurun_out/${T}_{v}_{r}.json"))
        print(r, v, "C3 %.2f (acct %.2f)" % (d["ms_per_step"], d["kernel_accounting"]["ms_per_step"]),
              "C4 %.3f" % d["fitc"]["C4"]["ms_per_step"], "C5 %.2f" % d["fitc"]["C5"]["ms_per_step"],
              "dag %.3f" % d["kernels_per_step"]["potrf_dag"]["ms"])
PY
