// Cross-workgroup handoff latency on MI355X: two resident workgroups ping-pong a counter through
// device-scope release/acquire atomics in global memory — the per-dependency cost a persistent
// (single-launch) factorisation would pay instead of a kernel boundary (~5-6 µs between dependent
// launches in the factorisation's graph, tools/gap_summary.py).  Pairs on the same XCD (blocks 0
// and 8 under round-robin dispatch) and on different XCDs (blocks 0 and 1).  Every spin is
// bounded, so a lost partner ends the kernel instead of hanging it.
//   hipcc -O3 --offload-arch=gfx950 tools/flag_latency.hip -o /tmp/fl && /tmp/fl
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kIters = 20000;
constexpr long kSpinMax = 1L << 22;

__device__ __forceinline__ int load_acq(int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_rel(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// grid of `nblk` workgroups; blocks a and b play, the others exit at once
__global__ void pingpong(int* flags, int a, int b, long long* cycles, int* fails) {
  const int me = blockIdx.x;
  if (me != a && me != b) return;
  int* ping = flags;       // written by a
  int* pong = flags + 64;  // written by b (separate 256-byte lines)
  if (threadIdx.x != 0) return;
  const long long t0 = clock64();
  int bad = 0;
  for (int i = 1; i <= kIters && !bad; ++i) {
    if (me == a) {
      store_rel(ping, i);
      long s = 0;
      while (load_acq(pong) != i && ++s < kSpinMax) __builtin_amdgcn_s_sleep(0);
      bad = s >= kSpinMax;
    } else {
      long s = 0;
      while (load_acq(ping) != i && ++s < kSpinMax) __builtin_amdgcn_s_sleep(0);
      bad = s >= kSpinMax;
      store_rel(pong, i);
    }
  }
  if (me == a) {
    cycles[0] = clock64() - t0;
    fails[0] = bad;
  }
}

int main() {
  int *flags, *fails;
  long long* cycles;
  hipMalloc(&flags, 256 * sizeof(int));
  hipMalloc(&fails, sizeof(int));
  hipMalloc(&cycles, sizeof(long long));
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const struct { const char* name; int a, b; } cases[] = {
      {"different XCDs (blocks 0, 1)", 0, 1}, {"same XCD (blocks 0, 8)", 0, 8},
      {"different XCDs (blocks 0, 5)", 0, 5}};
  for (const auto& c : cases) {
    hipMemset(flags, 0, 256 * sizeof(int));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, flags, c.a, c.b, cycles, fails);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long cyc = 0;
    int f = 0;
    hipMemcpy(&cyc, cycles, sizeof(cyc), hipMemcpyDeviceToHost);
    hipMemcpy(&f, fails, sizeof(f), hipMemcpyDeviceToHost);
    printf("%-32s round trip %.3f us (wall), %.0f clock64 ticks%s\n", c.name, 1e3 * ms / kIters,
           (double)cyc / kIters, f ? "  [a spin timed out]" : "");
  }
  printf("(clock rate attribute %d kHz)\n", clk_khz);
  return 0;
}
