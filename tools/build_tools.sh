#!/bin/bash
# Builds the standalone GPU probes used by the A/B scripts into tbin/ (git-ignored; it travels to
# the GPU box with gpurun, unlike ab/).  Cross-compiles here: hipcc --offload-arch=gfx950.
set -e
cd "$(dirname "$0")/.."
C=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc
mkdir -p tbin
F="-O3 --offload-arch=gfx950 -std=c++17 -I include -I $C -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1"
/opt/rocm/bin/hipcc $F tools/dag_bench.cpp -o tbin/dag_bench &
G=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/gpscore
/opt/rocm/bin/hipcc $F tools/gemm_bench.cpp -L $G -lgpscore -Wl,-rpath,'$ORIGIN/../'$G -o tbin/gemm_bench &
wait
/opt/rocm/bin/hipcc $F tools/gram_bench.cpp -o tbin/gram_bench
