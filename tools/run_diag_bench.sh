#!/bin/bash
# Leaf kernel (128×128 potrf + inverse): correctness vs a CPU Cholesky + timing, the library's
# MFMA leaf against the round-1 v3 kernel on the same box.
set -e
C=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc
F="-O3 --offload-arch=gfx950 -std=c++17 -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 -Wno-unused-value"
hipcc $F -I$C -Itools tools/diag_bench.cpp -o /tmp/db
for rep in 1 2; do timeout -k 5 60 /tmp/db "$@"; done
