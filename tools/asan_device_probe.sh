#!/bin/bash
# the host-ASan device pass (tests/test_asan.py) run by hand with its stderr kept, to see where
# the ASan runtime's HSA allocation interceptor runs out of memory on some boxes.
# ASAN_FIRST: libraries preloaded ahead of the ASan runtime (e.g. libhsa-runtime64, so that HIP
# binds the real hsa_amd_memory_pool_allocate; needs ASAN_EXTRA=verify_asan_link_order=0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so
P=scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd
LD_PRELOAD="${ASAN_FIRST:+$ASAN_FIRST }$RT${LD_PRELOAD:+ $LD_PRELOAD}" ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:verbosity=${ASAN_VERB:-0}${ASAN_EXTRA:+:$ASAN_EXTRA}" \
  GPSCORE_LIB=$PWD/$P/gpscore/libgpscore_asan.so timeout -k 10 240 python -u tools/asan_check.py device \
  > gpurun_out/asan_dev_${TAG:-x}.out 2> gpurun_out/asan_dev_${TAG:-x}.err
echo "asan device pass exit $?"
tail -c 3000 gpurun_out/asan_dev_${TAG:-x}.err
