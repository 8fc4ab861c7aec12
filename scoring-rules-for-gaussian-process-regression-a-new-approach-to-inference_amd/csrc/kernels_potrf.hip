// Diagonal-block kernel of the blocked Cholesky (replaces LAPACK ?potrf behind
// torch.potrf, KF:26 / KF:332).  One 1024-thread workgroup holds a whole
// 128×128 fp64 block in LDS (136 KiB of the CU's 160 KiB) and
//   1. factors it A = L Lᵀ (right-looking, one barrier per column; the
//      column is kept unscaled during the sweep and scaled once at the end),
//   2. records log L_ii (the ½log|A| terms of KF:332) and the first
//      non-positive pivot (torch.potrf's "leading minor not PD" error),
//   3. inverts L in place (LAPACK trti2 order: columns right to left,
//      x = -L_jj⁻¹ · L⁻¹[j+1:, j+1:] · L[j+1:, j]),
//   4. writes L⁻¹ with explicit zeros above the diagonal.
// Thread layout: 8 consecutive lanes own one row (16 waves × 8 rows); a row's
// partial dot products are combined with in-wave xor shuffles.  LDS row stride
// 136 doubles (≡ 16 dwords mod 64) keeps the 4-row × 8-column lane footprint of
// a ds_read_b64 conflict-free.
#include "gps_internal.h"

namespace gps {

constexpr int NB = 128;
constexpr int SL = 136;

__global__ __launch_bounds__(1024) void potrf_diag_kernel(const double* __restrict__ A, int64_t lda,
                                                          double* __restrict__ Linv, int64_t ldl,
                                                          double* __restrict__ Lout, int64_t ldlo,
                                                          double* __restrict__ logdiag, int* info,
                                                          int base, int nreal) {
  __shared__ __attribute__((aligned(16))) double a[NB * SL];
  __shared__ double sq[NB];
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB / 2; e += 1024) {
    const int r = e >> 6, c = (e & 63) * 2;
    const double2 v = *reinterpret_cast<const double2*>(A + (int64_t)r * lda + c);
    *reinterpret_cast<double2*>(&a[r * SL + c]) = v;
  }
  __syncthreads();

  const int i = tid >> 3, c = tid & 7;
  // ---- 1. unscaled right-looking factorisation: a[i][k] -= a[i][j] a[k][j] / d_j
  for (int j = 0; j < NB - 1; ++j) {
    if (i > j) {
      const double f = a[i * SL + j] / a[j * SL + j];
      for (int k = j + 1 + c; k <= i; k += 8) a[i * SL + k] = fma(-f, a[k * SL + j], a[i * SL + k]);
    }
    __syncthreads();
  }
  // ---- 2. pivots, log-diagonal, PD check
  if (tid < NB) {
    const double dj = a[tid * SL + tid];
    if (!(dj > 0.0) && tid < nreal) atomicMin(info, base + tid + 1);
    const double sj = sqrt(dj);
    sq[tid] = sj;
    logdiag[tid] = log(sj);
  }
  __syncthreads();
  for (int k = c; k <= i; k += 8) a[i * SL + k] /= sq[k];
  __syncthreads();
  if (Lout) {
    for (int e = tid; e < NB * NB; e += 1024) {
      const int r = e >> 7, cc = e & 127;
      Lout[(int64_t)r * ldlo + cc] = cc <= r ? a[r * SL + cc] : 0.0;
    }
  }
  // ---- 3. in-place inverse, columns right to left
  for (int j = NB - 1; j >= 0; --j) {
    double s = 0.0;
    if (i > j)
      for (int k = j + 1 + c; k <= i; k += 8) s = fma(a[i * SL + k], a[k * SL + j], s);
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    const double ljj = a[j * SL + j];
    __syncthreads();
    if (i > j && c == 0) a[i * SL + j] = -s / ljj;
    if (tid == 0) a[j * SL + j] = 1.0 / ljj;
    __syncthreads();
  }
  // ---- 4. write L⁻¹ (lower, explicit zeros above the diagonal)
  for (int e = tid; e < NB * NB; e += 1024) {
    const int r = e >> 7, cc = e & 127;
    Linv[(int64_t)r * ldl + cc] = cc <= r ? a[r * SL + cc] : 0.0;
  }
}

hipError_t launch_potrf_diag(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                             int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                             hipStream_t s) {
  if ((lda & 1) || (ldl & 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(1024), 0, s, A, lda, Linv, ldl, Lout, ldlo,
                     logdiag, info, base, nreal);
  return hipGetLastError();
}

}  // namespace gps
