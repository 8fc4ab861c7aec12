// Objective surfaces over a (length-scale, noise) grid — contour-plot.R (CP.R) restated for
// the GPU: thousands of independent small full GPs, one wavefront per grid point.
//
// Per point (ℓ_j, s_i):  A = sf²·exp(−½‖x − x'‖²/ℓ²) + s²I  (CP.R:15-23 rbf with k² = sf², the
// noise s.d. s entering as s², CP.R:45), in LDS.  Right-looking Cholesky, then L⁻¹ in place
// (LAPACK trti2 order), then  d = diag(A⁻¹) (column sums of L⁻¹∘L⁻¹), β = L⁻¹y, α = L⁻ᵀβ.
// From those, every CP.R objective:
//   LOO-CRPS   CP.R:43-53  μ = y − α/d, c = 1/d                         (R&W 5.12)
//   "wrong"    CP.R:55-64  in-sample predictive  μ = K A⁻¹y = y − s²α,
//                          c = diag(s²I + K − K A⁻¹K) = 2s² − s⁴d      (K = A − s²I)
//   NLML       CP.R:68-73  ½yᵀα + ½log|A| + ½n log 2π
//   LOO-LogS   CP.R:75-85  μ as LOO-CRPS, c = 1/d + s² (CP.R:81 adds the noise variance to the
//                          LOO variance; without the flag c = 1/d, the KF:416-424 form)
// n ≤ 128: A (n × (n+1) doubles) plus β in dynamic LDS.  A non-PD point (d_k ≤ 0) gives NaN
// objectives for that point (R's chol would stop the script; the grid keeps going).
#include <mutex>
#include <set>

#include "gps_internal.h"

namespace gps {

namespace {

__global__ __launch_bounds__(64) void surface_kernel(SurfaceParams p) {
  extern __shared__ double sm[];
  const int n = p.n, lda = n + 1;
  double* A = sm;                 // row-major, lower triangle used
  double* beta = sm + n * lda;    // β = L⁻¹y
  const int lane = threadIdx.x;
  const int gj = blockIdx.x % p.nl, gi = blockIdx.x / p.nl;
  const double ell = p.ell[gj], s = p.sd[gi], s2 = s * s;
  const double il2 = 1.0 / (ell * ell);
  // ---- A = K + s²I (lower)
  for (int i = lane; i < n; i += 64)
    for (int j = 0; j <= i; ++j) {
      double r2 = 0.0;
      for (int k = 0; k < p.d; ++k) {
        const double df = p.x[(int64_t)i * p.d + k] - p.x[(int64_t)j * p.d + k];
        r2 = fma(df, df, r2);
      }
      A[i * lda + j] = p.sf2 * exp(-0.5 * r2 * il2) + (i == j ? s2 : 0.0);
    }
  __syncthreads();
  // ---- Cholesky, right-looking: column k scaled, trailing lower part updated
  double half_logdet = 0.0;
  for (int k = 0; k < n; ++k) {
    const double dk = A[k * lda + k];
    const double inv = rsqrt(dk);  // d_k <= 0: NaN, propagates to every objective
    half_logdet += log(dk * inv);
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
      if (i > k) A[i * lda + k] *= inv;
      else if (i == k) A[k * lda + k] = dk * inv;
    }
    __syncthreads();
    for (int i = lane; i < n; i += 64)
      if (i > k) {
        const double li = A[i * lda + k];
        for (int j = k + 1; j <= i; ++j) A[i * lda + j] = fma(-li, A[j * lda + k], A[i * lda + j]);
      }
    __syncthreads();
  }
  // ---- X = L⁻¹ in place, column j from the right: X_ij = −(Σ_{k=j+1..i} X_ik L_kj) / L_jj
  for (int j = n - 1; j >= 0; --j) {
    const double ljj = A[j * lda + j];
    double t[2] = {0.0, 0.0};
    for (int q = 0; q < 2; ++q) {
      const int i = lane + 64 * q;
      if (i > j && i < n)
        for (int k = j + 1; k <= i; ++k) t[q] = fma(A[i * lda + k], A[k * lda + j], t[q]);
    }
    __syncthreads();  // every read of column j (L) before it is overwritten with X
    for (int q = 0; q < 2; ++q) {
      const int i = lane + 64 * q;
      if (i > j && i < n) A[i * lda + j] = -t[q] / ljj;
      else if (i == j) A[j * lda + j] = 1.0 / ljj;
    }
    __syncthreads();
  }
  // ---- β = L⁻¹y (row i), then α = L⁻ᵀβ and d = diag(A⁻¹) (column j)
  double quad = 0.0;
  for (int i = lane; i < n; i += 64) {
    double b = 0.0;
    for (int j = 0; j <= i; ++j) b = fma(A[i * lda + j], p.y[j], b);
    beta[i] = b;
    quad = fma(b, b, quad);
  }
  __syncthreads();
  double v[3] = {0.0, 0.0, 0.0};  // Σ LOO-CRPS, Σ in-sample CRPS, Σ LOO-LogS
  for (int j = lane; j < n; j += 64) {
    double a = 0.0, dj = 0.0;
    for (int i = j; i < n; ++i) {
      const double xij = A[i * lda + j];
      a = fma(xij, beta[i], a);
      dj = fma(xij, xij, dj);
    }
    const double y = p.y[j];
    const double mu = y - a / dj, c = 1.0 / dj;
    v[0] += crps_term(mu, c, y);
    v[1] += crps_term(y - s2 * a, 2.0 * s2 - s2 * s2 * dj, y);
    v[2] += logs_term(mu, p.logs_add_noise ? c + s2 : c, y);
  }
  quad = wave_sum(quad);
#pragma unroll
  for (int q = 0; q < 3; ++q) v[q] = wave_sum(v[q]);
  if (lane == 0) {
    const int64_t g = (int64_t)gi * p.nl + gj, st = (int64_t)p.ns * p.nl;
    p.out[g] = v[0] / n;
    p.out[st + g] = v[1] / n;
    p.out[2 * st + g] = 0.5 * quad + half_logdet + 0.5 * n * 1.83787706640934548356;
    p.out[3 * st + g] = v[2] / n;
  }
}

}  // namespace

size_t surface_lds_bytes(int n) { return (size_t)(n * (n + 1) + n) * sizeof(double); }

hipError_t launch_surface(const SurfaceParams& p, hipStream_t s) {
  if (p.n < 1 || p.n > GPS_SURFACE_MAX_N || p.d < 1 || p.nl < 1 || p.ns < 1)
    return hipErrorInvalidValue;
  const size_t lds = surface_lds_bytes(p.n);
  // the dynamic-LDS limit (133 KB at n = 128) is a per-device function attribute: set once per
  // device under a lock, so contexts on several threads or devices never race on it
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    static std::mutex mu;
    static std::set<int> done;
    std::lock_guard<std::mutex> lk(mu);
    if (!done.count(dev)) {
      e = hipFuncSetAttribute((const void*)surface_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)surface_lds_bytes(GPS_SURFACE_MAX_N));
      if (e != hipSuccess) return e;
      done.insert(dev);
    }
  }
  hipLaunchKernelGGL(surface_kernel, dim3((unsigned)(p.nl * p.ns)), dim3(64), lds, s, p);
  return hipGetLastError();
}

}  // namespace gps
