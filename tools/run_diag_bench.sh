#!/bin/bash
# Diagonal-block kernel: correctness vs a CPU Cholesky + timing (production v3, v1, v3 ablations).
set -e
C=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc
F="-O3 --offload-arch=gfx950 -std=c++17 -I$C -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 -Wno-unused-value"
hipcc $F tools/diag_bench.cpp -o /tmp/db_v3
hipcc $F -DGPS_DIAG_V1 tools/diag_bench.cpp -o /tmp/db_v1
echo "== v3"; timeout -k 5 60 /tmp/db_v3
echo "== v1"; timeout -k 5 60 /tmp/db_v1
if [ "$1" = "ablate" ]; then
  for m in 1 2 3 4 5; do
    hipcc $F -DGPS_V3_ABLATE=$m tools/diag_bench.cpp -o /tmp/db_a$m
    echo "== v3 ablate $m"; timeout -k 5 60 /tmp/db_a$m | grep "us per"
  done
fi
