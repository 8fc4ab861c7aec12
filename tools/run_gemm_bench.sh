#!/bin/bash
# build + run the GEMM microbenchmark on the GPU box (after the library is built)
#   tools/run_gemm_bench.sh          fixed cases
#   tools/run_gemm_bench.sh sweep    recursion-level shapes under every launch plan
set -e
P=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd
make -s -C $P/csrc -j16 >/dev/null
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$P/csrc -Iinclude tools/gemm_bench.cpp \
  -L$P/gpscore -lgpscore -Wl,-rpath,$PWD/$P/gpscore -o /tmp/gb 2>/dev/null
timeout -k 5 300 /tmp/gb "$@"
