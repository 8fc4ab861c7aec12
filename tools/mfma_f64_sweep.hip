// Sweep of f64 MFMA throughput vs waves/SIMD and independent accumulators, with the
// in-kernel shader clock (s_memtime / s_memrealtime @100 MHz) so cycles are real cycles.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, unsigned long long* clk, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){seed, seed, seed, seed};
  double a = seed + threadIdx.x * 1e-9, b = seed - threadIdx.x * 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int NACC>
void run(int bpc, int iters) {
  double* out; unsigned long long* clk;
  int blocks = 256 * bpc;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  hipMalloc(&clk, (size_t)blocks * 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1e-3);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1e-3);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  double ghz = (double)h[0] / h[1] * 0.1;
  double flops = (double)blocks * 4 * iters * NACC * 2048.0;
  double cyc = (double)h[0] / (iters * NACC * bpc);
  printf("NACC=%2d waves/SIMD=%d: %7.3f ms %6.2f TF  clock %.2f GHz  %.1f cyc/MFMA/SIMD (in-kernel)\n",
         NACC, bpc, ms, flops / ms / 1e9, ghz, cyc);
  hipFree(out); hipFree(clk);
}

int main() {
  int it = 40000;
  run<1>(1, it); run<2>(1, it / 2); run<4>(1, it / 4); run<8>(1, it / 8);
  run<1>(2, it); run<2>(2, it / 2); run<4>(2, it / 4); run<8>(2, it / 8);
  run<1>(4, it / 2); run<2>(4, it / 4); run<4>(4, it / 8);
  run<1>(8, it / 4); run<2>(8, it / 8);
  return 0;
}
