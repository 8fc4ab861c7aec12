#!/bin/bash
# Same-box A/B of a compile-time library variant: builds libgpscore with EXTRA=$1 into /tmp/var,
# runs the GEMM microbenchmark and the C3 headline against both libraries, interleaved.
#   bash tools/run_lib_variant_ab.sh -DGPS_SETPRIO   -> gpurun_out/var_*.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
P=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd
mkdir -p /tmp/var
make -s -C $P/csrc -j16 >/dev/null || exit 1
make -s -C $P/csrc -j16 GPS_BUILD_DIR=/tmp/var/build GPS_LIB_OUT=/tmp/var/libgpscore.so GPS_EXTRA_FLAGS="$1" >/dev/null || exit 1
for v in base var; do
  L=$PWD/$P/gpscore; [ $v = var ] && L=/tmp/var
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$P/csrc -Iinclude tools/gemm_bench.cpp \
    -L$L -lgpscore -Wl,-rpath,$L -o /tmp/gb_$v 2>/dev/null || exit 1
done
timeout -k 5 200 /tmp/gb_base layout > gpurun_out/var_gb_base.txt 2>&1 || exit 1
timeout -k 5 200 /tmp/gb_var layout > gpurun_out/var_gb_var.txt 2>&1 || exit 1
B="bench.py --steps 5 --warmup 2 --no-fitc --no-grad --no-block --no-cpu"
for r in 1 2; do
  timeout -k 5 200 python -u $B > gpurun_out/var_bench_base_$r.json 2>/dev/null || exit 1
  GPSCORE_LIB=/tmp/var/libgpscore.so timeout -k 5 200 python -u $B > gpurun_out/var_bench_var_$r.json 2>/dev/null || exit 1
done
echo ok
