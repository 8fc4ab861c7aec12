// f64 MFMA issue rate per SIMD vs waves per SIMD and independent accumulators (round 4): is the
// persistent kernel's one-wave-per-SIMD layout MFMA-issue-bound?  Distinct A/B registers per
// accumulator; clock from s_memtime vs s_memrealtime inside the kernel.
//   mfma_f64_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void rate(double* out, unsigned long long* clk, int iters, double seed) {
  d4 acc[NACC];
  double a[NACC], b[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    acc[i] = (d4){seed, seed, seed, seed};
    a[i] = seed + (threadIdx.x + i) * 1e-9;
    b[i] = seed - (threadIdx.x + 3 * i) * 1e-9;
  }
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[i], acc[i], 0, 0, 0);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }
}

template <int NACC>
void run(int threads, int blocks, int iters) {
  double* out; unsigned long long* clk;
  hipMalloc(&out, (size_t)blocks * threads * 8); hipMalloc(&clk, 16);
  rate<NACC><<<blocks, threads>>>(out, clk, iters, 1e-3);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  rate<NACC><<<blocks, threads>>>(out, clk, iters, 1e-3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double tflops = (double)blocks * (threads / 64) * iters * NACC * 2048.0 / (ms * 1e-3) / 1e12;
  unsigned long long h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double cyc = (double)h[0], us = h[1] / 100.0;
  const int waves_per_simd = (threads / 64 + 3) / 4;  // one block per CU (blocks = CUs)
  printf("NACC=%2d waves/SIMD=%d: %.1f shader cycles per MFMA per wave, SIMD issue every %.1f cycles "
         "(clock %.2f GHz); chip %.1f TF/s over %.3f ms\n", NACC, waves_per_simd, cyc / ((double)iters * NACC),
         cyc / ((double)iters * NACC * waves_per_simd), cyc / us / 1e3, tflops, ms);
  hipFree(out); hipFree(clk);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<1>(256, cus, 4000);
  run<2>(256, cus, 2000);
  run<4>(256, cus, 1000);
  run<8>(256, cus, 500);
  run<1>(512, cus, 4000);
  run<2>(512, cus, 2000);
  run<4>(512, cus, 1000);
  run<8>(512, cus, 500);
  run<4>(1024, cus, 1000);
  return 0;
}
