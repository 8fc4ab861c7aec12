// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate / dependent latency on gfx950,
// plus the fragment-map check (A = I, asymmetric B).
// (Its rate column is event-timed over blocks the dispatcher may pack two to a CU, so it
// reads ~2x slow; tools/mfma_f64_rate.hip measures per-wave cycles in-kernel: 64 per MFMA.)  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_f64_probe.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){seed, seed, seed, seed};
  double a = seed + threadIdx.x * 1e-9, b = seed - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void layout(const double* A, const double* B, double* C) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A[i][k], 16x4
  double b = B[(l >> 4) * 16 + (l & 15)];  // B[k][j], 4x16
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[l * 4 + r] = acc[r];
}

template <int NACC>
void run(int blocks_per_cu, int iters) {
  double* out;
  hipMalloc(&out, 256 * 8 * 256 * 8);
  int blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = (double)blocks * 4 * iters * NACC * 2048.0;
  double waves_per_simd = blocks_per_cu;  // 4 waves/block, 4 SIMDs/CU
  printf("NACC=%2d blocks/CU=%d: %.3f ms  %.2f TFLOP/s  (%.1f cycles/MFMA/SIMD @2.4GHz)\n", NACC,
         blocks_per_cu, ms, flops / ms / 1e9, ms * 1e-3 * 2.4e9 / (iters * NACC * waves_per_simd));
  hipFree(out);
}

int main() {
  double hA[64], hB[64], hC[256], *dA, *dB, *dC;
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) hA[i * 4 + k] = (i == k) ? 1.0 : 0.0;
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) hB[k * 16 + j] = 100 * k + j;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 2048);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r, col = l & 15;
    double expect = row < 4 ? 100 * row + col : 0.0;  // C = I(16x4) * B
    if (hC[l * 4 + r] != expect) bad++;
  }
  printf("f64 MFMA C map row=(l>>4)+4r col=l&15: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  run<1>(1, 20000);
  run<4>(1, 5000);
  run<8>(1, 2500);
  run<16>(1, 1250);
  run<16>(2, 1250);
  run<8>(2, 2500);
  return 0;
}
