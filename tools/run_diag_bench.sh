#!/bin/bash
# Diagonal-block kernel: correctness vs a CPU Cholesky + timing.
#   tools/run_diag_bench.sh            working copy vs the committed (HEAD) kernel, same box
#   tools/run_diag_bench.sh stamps     + per-phase s_memtime stamps of the working copy
#   tools/run_diag_bench.sh ablate     + ablations of the working copy
set -e
C=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc
F="-O3 --offload-arch=gfx950 -std=c++17 -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 -Wno-unused-value"
hipcc $F -I$C tools/diag_bench.cpp -o /tmp/db_cur
if [ -f tools/diag_head/kernels_potrf.hip ]; then
  mkdir -p /tmp/dhead && cp tools/diag_head/kernels_potrf.hip /tmp/dhead/ && cp $C/gps_internal.h /tmp/dhead/
  hipcc $F -I/tmp/dhead tools/diag_bench.cpp -o /tmp/db_head
fi
for rep in 1 2; do
  echo "== working copy"; timeout -k 5 60 /tmp/db_cur
  if [ -x /tmp/db_head ]; then echo "== HEAD"; timeout -k 5 60 /tmp/db_head; fi
done
if [ "$1" = "stamps" ]; then
  hipcc $F -I$C -DGPS_V3_STAMPS tools/diag_bench.cpp -o /tmp/db_st
  echo "== stamps (last launch)"; timeout -k 5 60 /tmp/db_st
fi
if [ "$1" = "ablate" ]; then
  for m in 1 2 3 4 5; do
    hipcc $F -I$C -DGPS_V3_ABLATE=$m tools/diag_bench.cpp -o /tmp/db_a$m
    echo "== ablate $m"; timeout -k 5 60 /tmp/db_a$m | grep "us per"
  done
fi
