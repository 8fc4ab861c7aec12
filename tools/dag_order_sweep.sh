#!/bin/bash
# sweep of the persistent factorisation's order-1 weights (LEAF,fine,TRSM,UPD,UPDX,FIN,hand-off)
# on dag_bench, one box; output: gpurun_out/dag_weights_<tag>.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/dag_weights_${TAG:-sweep}.txt
: > $out
for w in ${WEIGHTS:-35,6,9.7,11.7,11.2,9.3,2.5}; do
  for tn in ${SIZES:-20:256 16:128}; do  # T:workgroups
    timeout -k 10 60 ab/dag_bench ${tn/:/ } - ${REPS:-30} 3 1 1 0 $w 2>&1 | grep -v traced | sed 's/; max|XAX.*//' >> $out || exit 1
  done
done
echo done
