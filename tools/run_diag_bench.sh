#!/bin/bash
set -e
C=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc
for m in 0 1 2 3; do
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$C -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 \
    -DGPS_DIAG_ABLATE=$m tools/diag_bench.cpp -o /tmp/db$m 2>/dev/null
  timeout -k 5 60 /tmp/db$m
done
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$C -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 \
  -DGPS_DIAG_STAMPS tools/diag_bench.cpp -o /tmp/dbs 2>/dev/null
timeout -k 5 60 /tmp/dbs
