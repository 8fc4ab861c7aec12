#!/bin/bash
# build + run the GEMM microbenchmark on the GPU box (after the library is built)
set -e
P=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd
make -s -C $P/csrc -j16 >/dev/null
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$P/csrc -Iinclude tools/gemm_bench.cpp \
  -L$P/gpscore -lgpscore -Wl,-rpath,$PWD/$P/gpscore -o /tmp/gb 2>/dev/null
timeout -k 5 120 /tmp/gb
