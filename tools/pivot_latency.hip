// Cycle cost of the one-thread 4x4 Cholesky + inverse chain (the diag kernel's serial
// pivot path), with ocml rsqrt vs rsq+2 Newton, measured with s_memtime in one wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int MODE>
__global__ void piv(double* out, unsigned long long* cyc, int iters) {
  double a[4][4];
  for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) a[r][c] = (r == c ? 4.0 : 0.5) + 1e-3 * threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double acc = 0;
  for (int it = 0; it < iters; ++it) {
    double l[4][4], is[4];
    for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) l[r][c] = a[r][c];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double d = l[j][j];
      if (MODE == 0) is[j] = rsqrt(d);
      else if (MODE == 1) { double y = __builtin_amdgcn_rsq(d); double h = d * y * y; y = y * fma(-0.5, h, 1.5); h = d * y * y; is[j] = y * fma(-0.5, h, 1.5); }
      else is[j] = 1.0 / sqrt(d);
      l[j][j] = d * is[j];
#pragma unroll
      for (int r = j + 1; r < 4; ++r) l[r][j] *= is[j];
#pragma unroll
      for (int r = j + 1; r < 4; ++r)
#pragma unroll
        for (int c = j + 1; c <= r; ++c) l[r][c] = fma(-l[r][j], l[c][j], l[r][c]);
    }
    double x[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r < c) x[r][c] = 0.0;
        else if (r == c) x[r][c] = is[r];
        else { double t = 0.0;
#pragma unroll
          for (int k = c; k < r; ++k) t = fma(l[r][k], x[k][c], t);
          x[r][c] = -t * is[r]; }
      }
    acc += x[3][0] + l[3][3];
    a[0][0] += 1e-12 * x[3][0];  // loop-carried dependency
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  double* o; unsigned long long* c; hipMalloc(&o, 8 * 64); hipMalloc(&c, 8);
  const int it = 2000;
  for (int m = 0; m < 3; ++m) {
    unsigned long long h = 0;
    for (int rep = 0; rep < 2; ++rep) {
      if (m == 0) hipLaunchKernelGGL(piv<0>, dim3(1), dim3(64), 0, 0, o, c, it);
      if (m == 1) hipLaunchKernelGGL(piv<1>, dim3(1), dim3(64), 0, 0, o, c, it);
      if (m == 2) hipLaunchKernelGGL(piv<2>, dim3(1), dim3(64), 0, 0, o, c, it);
      hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    }
    printf("mode %d (%s): %.0f cycles per 4x4 factor+inverse\n", m, m == 0 ? "ocml rsqrt" : (m == 1 ? "rsq+2NR" : "1/sqrt"), (double)h / it);
  }
  return 0;
}
