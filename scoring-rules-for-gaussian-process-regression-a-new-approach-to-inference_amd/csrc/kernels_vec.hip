// Bandwidth / latency-bound kernels around the factorisation:
//   β = L⁻¹y (row GEMV), α = L⁻ᵀβ and diag(A⁻¹) = colsum(L⁻¹∘L⁻¹) (one fused column
//   pass), the LOO closed form (R&W eq. 5.12, KF:241-244), the FITC Λ and LOO
//   terms (K20:225-232 restated), and the scoring-rule sums crps / logs /
//   trivial_loss / SMSE / MSE / ±2σ coverage (KF:52-68, 110-134, 276-292).
// All reductions are fixed-order trees (no atomics) so results are bitwise
// reproducible run to run.
#include "gps_internal.h"

namespace gps {

// ------------------------------------------------------------------ GEMV rows
// one wave per row, 16-byte loads; tile-lower: k < (i/128 + 1)*128
__global__ __launch_bounds__(256) void gemv_rows_kernel(const double* __restrict__ M, int64_t ldm,
                                                        const double* __restrict__ x,
                                                        double* __restrict__ y, int rows, int cols,
                                                        int lower) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int kend = lower ? min(cols, (row / GPS_TILE + 1) * GPS_TILE) : cols;
  const double* r = M + (int64_t)row * ldm;
  double s0 = 0.0, s1 = 0.0;
  for (int k = 2 * lane; k < kend; k += 128) {
    const double2 v = *reinterpret_cast<const double2*>(r + k);
    const double2 xv = *reinterpret_cast<const double2*>(x + k);
    s0 = fma(v.x, xv.x, s0);
    s1 = fma(v.y, xv.y, s1);
  }
  const double s = wave_sum(s0 + s1);
  if (lane == 0) y[row] = s;
}

hipError_t launch_gemv_lower(const double* L, int64_t ldl, const double* x, double* y, int n_pad,
                             hipStream_t s) {
  hipLaunchKernelGGL(gemv_rows_kernel, dim3((n_pad + 3) / 4), dim3(256), 0, s, L, ldl, x, y, n_pad,
                     n_pad, 1);
  return hipGetLastError();
}
hipError_t launch_gemv_full(const double* M, int64_t ldm, const double* x, double* y, int rows,
                            int cols, hipStream_t s) {
  if (cols & 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gemv_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, M, ldm, x, y, rows,
                     cols, 0);
  return hipGetLastError();
}

// ------------------------------------------------------- column reductions
constexpr int CR_ROWS = 256;  // rows per chunk
constexpr int CR_COLS = 512;  // columns per block (2 per thread)

__global__ __launch_bounds__(256) void colred_kernel(const double* __restrict__ M, int64_t ldm,
                                                     int rows, int cols, int lower, int crows,
                                                     const double* __restrict__ w,
                                                     const double* __restrict__ rowscale,
                                                     double* __restrict__ slab1,
                                                     double* __restrict__ slab2) {
  const int c = blockIdx.x * CR_COLS + 2 * threadIdx.x;
  const int chunk = blockIdx.y;
  if (c >= cols) return;
  int r0 = chunk * crows, r1 = min(rows, r0 + crows);
  if (lower) r0 = max(r0, (c / GPS_TILE) * GPS_TILE);
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  // (unrolled so 8 rows' loads are in flight ahead of the in-order FMAs: one memory latency
  // per 8 rows instead of per row — the m×m passes of the FITC path have only a few chunks)
#pragma unroll 8
  for (int r = r0; r < r1; ++r) {
    double2 v = *reinterpret_cast<const double2*>(M + (int64_t)r * ldm + c);
    if (rowscale) {
      const double sc = rowscale[r];
      v.x *= sc;
      v.y *= sc;
    }
    if (slab1) {
      const double wr = w[r];
      a0 = fma(v.x, wr, a0);
      a1 = fma(v.y, wr, a1);
    }
    b0 = fma(v.x, v.x, b0);
    b1 = fma(v.y, v.y, b1);
  }
  const int64_t o = (int64_t)chunk * cols + c;
  if (slab1) *reinterpret_cast<double2*>(slab1 + o) = make_double2(a0, a1);
  if (slab2) *reinterpret_cast<double2*>(slab2 + o) = make_double2(b0, b1);
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const double* __restrict__ slab, int64_t ld,
                                                       int nslab, int64_t len,
                                                       const double* __restrict__ init,
                                                       double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= len) return;
  double s = init ? init[j] : 0.0;
  // (8 slabs' loads in flight ahead of the in-order adds: the predictive pass sums 157 slabs,
  // one memory latency each without the unroll)
#pragma unroll 8
  for (int q = 0; q < nslab; ++q) s += slab[(int64_t)q * ld + j];
  out[j] = s;
}

hipError_t launch_slab_sum(const double* slab, int64_t ld, int nslab, int64_t len,
                           const double* init, double* out, hipStream_t s) {
  if (len <= 0) return hipSuccess;
  hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, slab,
                     ld, nslab, len, init, out);
  return hipGetLastError();
}

hipError_t launch_colred(const double* M, int64_t ldm, int rows, int cols, int lower,
                         const double* w, const double* rowscale, double* s1, double* s2,
                         double* slab, hipStream_t s, int crows) {
  if ((cols & 1) || (ldm & 1) || crows < 1) return hipErrorInvalidValue;
  const int nchunk = (rows + crows - 1) / crows;
  double* slab1 = s1 ? slab : nullptr;
  double* slab2 = s2 ? slab + (int64_t)nchunk * cols : nullptr;
  hipLaunchKernelGGL(colred_kernel, dim3((cols + CR_COLS - 1) / CR_COLS, nchunk), dim3(256), 0, s,
                     M, ldm, rows, cols, lower, crows, w, rowscale, slab1, slab2);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (s1 && (e = launch_slab_sum(slab1, cols, nchunk, cols, nullptr, s1, s)) != hipSuccess) return e;
  if (s2 && (e = launch_slab_sum(slab2, cols, nchunk, cols, nullptr, s2, s)) != hipSuccess) return e;
  return hipSuccess;
}

// the column pass alone: chunk partials of Σ w_r M_rc (slab) and Σ M_rc² (slab + nchunk·cols);
// returns the chunk count (the caller sums the chunks, e.g. fused into its row finaliser)
int launch_colred_partials(const double* M, int64_t ldm, int rows, int cols, int lower,
                           const double* w, double* slab, hipStream_t s) {
  if ((cols & 1) || (ldm & 1)) return -1;
  const int nchunk = (rows + CR_ROWS - 1) / CR_ROWS;
  hipLaunchKernelGGL(colred_kernel, dim3((cols + CR_COLS - 1) / CR_COLS, nchunk), dim3(256), 0, s,
                     M, ldm, rows, cols, lower, CR_ROWS, w, nullptr, slab, slab + (int64_t)nchunk * cols);
  return hipGetLastError() == hipSuccess ? nchunk : -1;
}

// sum split-K slabs of a symmetric M×M accumulator; tile-lower kept, strict-upper
// tiles zeroed (so the buffer can be all-reduced / factorised as is)
__global__ __launch_bounds__(256) void sym_slab_sum_kernel(const double* __restrict__ slab,
                                                           int64_t stride, int nslab, int M,
                                                           const double* __restrict__ base,
                                                           double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * M) return;
  const int i = (int)(e / M), j = (int)(e - (int64_t)i * M);
  double v = 0.0;
  if (j / GPS_TILE <= i / GPS_TILE) {
    for (int q = 0; q < nslab; ++q) v += slab[(int64_t)q * stride + e];
    if (base) v = base[e] + v;  // base + (Σ slabs): the sum, then the base, as two launches would
  }
  dst[e] = v;
}

hipError_t launch_sym_slab_sum(const double* slab, int64_t slice_stride, int nslab, int M,
                               const double* base, double* dst, hipStream_t s) {
  const int64_t tot = (int64_t)M * M;
  hipLaunchKernelGGL(sym_slab_sum_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     slab, slice_stride, nslab, M, base, dst);
  return hipGetLastError();
}

// Lower-packed form of a symmetric m×m accumulator (row i holds columns 0..i at offset
// i(i+1)/2): the payload of the FITC row-shard all-reduce, m(m+1)/2 doubles instead of
// the padded m_pad².  Pack sums the split-K slabs in slice order (the
// same sums sym_slab_sum forms); unpack adds the optional base and writes either the
// lower 128-tiles (strict-upper tiles zero, as sym_slab_sum) or the full symmetric matrix.
// packed elements [e0, e1) of the lower-packed (row-major) sum of the slabs: a row block of B
// (rows [r0, r1) are elements [r0(r0+1)/2, r1(r1+1)/2)) can be packed as soon as its tiles exist
__global__ __launch_bounds__(256) void sym_pack_kernel(const double* __restrict__ slab,
                                                       int64_t stride, int nslab, int64_t e0,
                                                       int64_t e1, int M,
                                                       double* __restrict__ packed) {
  const int64_t e = e0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= e1) return;
  int i = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
  while ((int64_t)(i + 1) * (i + 2) / 2 <= e) ++i;
  while ((int64_t)i * (i + 1) / 2 > e) --i;
  const int j = (int)(e - (int64_t)i * (i + 1) / 2);
  const int64_t src = (int64_t)i * M + j;
  double v = 0.0;
  for (int q = 0; q < nslab; ++q) v += slab[(int64_t)q * stride + src];
  packed[e] = v;
}

__global__ __launch_bounds__(256) void sym_unpack_kernel(const double* __restrict__ packed, int m,
                                                         int M, const double* __restrict__ base,
                                                         int full, double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * M) return;
  const int i = (int)(e / M), j = (int)(e - (int64_t)i * M);
  double v = 0.0;
  if (full || j / GPS_TILE <= i / GPS_TILE) {
    if (i < m && j < m) {
      const int hi = i > j ? i : j, lo = i > j ? j : i;
      v = packed[(int64_t)hi * (hi + 1) / 2 + lo];
    }
    if (base) v += base[e];
  }
  dst[e] = v;
}

hipError_t launch_sym_pack(const double* slab, int64_t slice_stride, int nslab, int r0, int r1,
                           int M, double* packed, hipStream_t s) {
  const int64_t e0 = (int64_t)r0 * (r0 + 1) / 2, e1 = (int64_t)r1 * (r1 + 1) / 2;
  if (r1 <= r0) return hipSuccess;
  hipLaunchKernelGGL(sym_pack_kernel, dim3((unsigned)((e1 - e0 + 255) / 256)), dim3(256), 0, s,
                     slab, slice_stride, nslab, e0, e1, M, packed);
  return hipGetLastError();
}

hipError_t launch_sym_unpack(const double* packed, int m, int M, const double* base, int full,
                             double* dst, hipStream_t s) {
  const int64_t tot = (int64_t)M * M;
  hipLaunchKernelGGL(sym_unpack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     packed, m, M, base, full, dst);
  return hipGetLastError();
}

// ------------------------------------------------------ two-level row sums
// The row finalisers below run one thread per row over many workgroups (a single workgroup
// walking 40k-200k rows took 30-105 µs of a FITC unit's critical path); each workgroup writes
// its block_sum partials to part[block·NV + q] and this one-workgroup kernel adds them in block
// order through a fixed tree — deterministic, like every reduction here.
template <int NV>
__global__ __launch_bounds__(1024) void partials_sum_kernel(const double* __restrict__ part,
                                                            int nblk, double* __restrict__ out) {
  __shared__ double sh[NV * 16];
  double v[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 1024)
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] += part[(int64_t)b * NV + q];
  block_sum<NV>(v, sh);
  if (threadIdx.x == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) out[q] = v[q];
}

// ------------------------------------------------------------ full-GP LOO
// α_i = Σ_t slab1[t][i] and d_i = Σ_t slab2[t][i] (the column pass's chunk partials, summed in
// chunk order as slab_sum_kernel does), stored, then the LOO closed form (R&W 5.12, KF:241-244)
// per row; per-workgroup partials [Σ crps, Σ logs, Σ log L_ii, Σ β²] (pads carry zeros)
__global__ __launch_bounds__(256) void full_loo_rows_kernel(
    const double* __restrict__ y, const double* __restrict__ slab1, const double* __restrict__ slab2,
    int64_t ld, int nslab, const double* __restrict__ beta, const double* __restrict__ logdiag,
    int n, int n_pad, double* __restrict__ alpha, double* __restrict__ dinv,
    double* __restrict__ mu_loo, double* __restrict__ var_loo, double* __restrict__ part) {
  __shared__ double sh[4 * 16];
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n_pad) {
    double a = 0.0, dd = 0.0;
#pragma unroll 8
    for (int t = 0; t < nslab; ++t) {
      a += slab1[(int64_t)t * ld + i];
      dd += slab2[(int64_t)t * ld + i];
    }
    alpha[i] = a;
    dinv[i] = dd;
    v[2] = logdiag[i];
    v[3] = beta[i] * beta[i];
    if (i < n) {
      const double m = y[i] - a / dd;
      const double c = 1.0 / dd;
      mu_loo[i] = m;
      var_loo[i] = c;
      v[0] = crps_term(m, c, y[i]);
      v[1] = logs_term(m, c, y[i]);
    }
  }
  block_sum<4>(v, sh);
  if (threadIdx.x == 0)
    for (int q = 0; q < 4; ++q) part[(int64_t)blockIdx.x * 4 + q] = v[q];
}
// obj: [nlml, loo_crps, loo_logs, logdet, quad] from the sums [Σcrps, Σlogs, Σlog L_ii, Σβ²]
__global__ void full_loo_obj_kernel(const double* __restrict__ sums, int n, double* __restrict__ obj) {
  if (threadIdx.x != 0) return;
  const double logdet = 2.0 * sums[2], quad = sums[3];
  obj[0] = 0.5 * n * 1.83787706640934548356 + 0.5 * logdet + 0.5 * quad;
  obj[1] = sums[0] / n;
  obj[2] = sums[1] / n;
  obj[3] = logdet;
  obj[4] = quad;
}

hipError_t launch_full_loo(const double* y, const double* slab, int nslab, int64_t ld,
                           const double* beta, const double* logdiag, int n, double* alpha,
                           double* dinv, double* mu_loo, double* var_loo, double* obj,
                           double* part, hipStream_t s) {
  const int n_pad = (int)pad_to(n);
  const int nblk = n_pad / 256 + (n_pad % 256 ? 1 : 0);
  hipLaunchKernelGGL(full_loo_rows_kernel, dim3(nblk), dim3(256), 0, s, y, slab,
                     slab + (int64_t)nslab * ld, ld, nslab, beta, logdiag, n, n_pad, alpha, dinv,
                     mu_loo, var_loo, part);
  hipLaunchKernelGGL(partials_sum_kernel<4>, dim3(1), dim3(1024), 0, s, part, nblk, obj + 8);
  hipLaunchKernelGGL(full_loo_obj_kernel, dim3(1), dim3(64), 0, s, obj + 8, n, obj);
  return hipGetLastError();
}

// CP.R surface point from a resident fit (n > GPS_SURFACE_MAX_N): the "wrong" in-sample CRPS
// (CP.R:55-64: μ = y − s²α, c = 2s² − s⁴ d) and the LOO-LogS with CP.R:81's + s² (or not),
// from α and d = diag(A⁻¹) — the surface kernel's formulas (kernels_surface.hip)
__global__ __launch_bounds__(256) void surface_point_rows_kernel(
    const double* __restrict__ y, const double* __restrict__ alpha, const double* __restrict__ dinv,
    int n, double s2, int add_noise, double* __restrict__ part) {
  __shared__ double sh[2 * 16];
  double v[2] = {0.0, 0.0};
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const double a = alpha[i], dj = dinv[i], yi = y[i];
    const double mu = yi - a / dj, c = 1.0 / dj;
    v[0] = crps_term(yi - s2 * a, 2.0 * s2 - s2 * s2 * dj, yi);
    v[1] = logs_term(mu, add_noise ? c + s2 : c, yi);
  }
  block_sum<2>(v, sh);
  if (threadIdx.x == 0) {
    part[(int64_t)blockIdx.x * 2] = v[0];
    part[(int64_t)blockIdx.x * 2 + 1] = v[1];
  }
}
hipError_t launch_surface_point_sums(const double* y, const double* alpha, const double* dinv,
                                     int n, double s2, int add_noise, double* sums, double* part,
                                     hipStream_t s) {
  const int nblk = std::max(1, (n + 255) / 256);
  hipLaunchKernelGGL(surface_point_rows_kernel, dim3(nblk), dim3(256), 0, s, y, alpha, dinv, n, s2,
                     add_noise, part);
  hipLaunchKernelGGL(partials_sum_kernel<2>, dim3(1), dim3(1024), 0, s, part, nblk, sums);
  return hipGetLastError();
}

// --------------------------------------------------------------- predictive
__global__ __launch_bounds__(256) void pred_finalize_kernel(const double* __restrict__ s1,
                                                            const double* __restrict__ s2, int nt,
                                                            double base_var, double* __restrict__ mu,
                                                            double* __restrict__ var) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= nt) return;
  mu[j] = s1[j];
  var[j] = base_var - s2[j];
}
hipError_t launch_pred_finalize(const double* s1, const double* s2, int nt, double base_var,
                                double* mu, double* var, hipStream_t s) {
  hipLaunchKernelGGL(pred_finalize_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, s1, s2, nt,
                     base_var, mu, var);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void fitc_pred_finalize_kernel(const double* __restrict__ qm,
                                                                 const double* __restrict__ qb,
                                                                 int nt, double base_var,
                                                                 double* __restrict__ var) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= nt) return;
  var[j] = base_var - qm[j] + qb[j];
}
hipError_t launch_fitc_pred_finalize(const double* qm, const double* qb, int nt, double base_var,
                                     double* var, hipStream_t s) {
  hipLaunchKernelGGL(fitc_pred_finalize_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, qm, qb, nt,
                     base_var, var);
  return hipGetLastError();
}

// sums: [Σcrps, Σlogs, Σmsll, Σ(μ−y)², Σ(ȳtr−y)², Σcover]  (KF:276-292, 110-134)
__global__ __launch_bounds__(256) void score_rows_kernel(const double* __restrict__ mu,
                                                         const double* __restrict__ var,
                                                         const double* __restrict__ y, int nt,
                                                         double ytr_mean, double ytr_var,
                                                         double* __restrict__ part) {
  __shared__ double sh[6 * 16];
  double v[6] = {0, 0, 0, 0, 0, 0};
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < nt) {
    const double triv_c = 0.5 * log(6.28318530717958647692 * ytr_var);
    const double m = mu[j], c = var[j], t = y[j];
    v[0] = crps_term(m, c, t);
    const double ls = logs_term(m, c, t);
    v[1] = ls;
    const double e0 = t - ytr_mean;
    v[2] = ls - (triv_c + e0 * e0 / (2.0 * ytr_var));
    v[3] = (m - t) * (m - t);
    v[4] = e0 * e0;
    const double sd = sqrt(c);
    v[5] = ((m + 2.0 * sd - t) > 0.0 && (t - (m - 2.0 * sd)) > 0.0) ? 1.0 : 0.0;
  }
  block_sum<6>(v, sh);
  if (threadIdx.x == 0)
    for (int q = 0; q < 6; ++q) part[(int64_t)blockIdx.x * 6 + q] = v[q];
}
hipError_t launch_score_sums(const double* mu, const double* var, const double* y, int nt,
                             double ytr_mean, double ytr_var, double* sums, double* part,
                             hipStream_t s) {
  const int nblk = std::max(1, (nt + 255) / 256);
  hipLaunchKernelGGL(score_rows_kernel, dim3(nblk), dim3(256), 0, s, mu, var, y, nt, ytr_mean,
                     ytr_var, part);
  hipLaunchKernelGGL(partials_sum_kernel<6>, dim3(1), dim3(1024), 0, s, part, nblk, sums);
  return hipGetLastError();
}

// ---------------------------------------------------------------------- FITC
// q_i = Σ_t slab_t[i] (the row-norm GEMM's per-column-tile partials, summed in tile order as
// slab_sum_kernel does), then Λ: λ_i = sf2 − q_i + σ² (K20:225-228), 1/λ, y/λ; partial sums
// [Σ log λ, Σ y²/λ] per workgroup
__global__ __launch_bounds__(256) void fitc_lambda_rows_kernel(
    const double* __restrict__ slab, int64_t ld, int nslab, const double* __restrict__ y, int n,
    int n_pad, double sf2, double sn2, double* __restrict__ q, double* __restrict__ lam,
    double* __restrict__ inv_lam, double* __restrict__ ys, double* __restrict__ part) {
  __shared__ double sh[2 * 16];
  double v[2] = {0.0, 0.0};
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n_pad) {
    double qi = 0.0;
#pragma unroll 8
    for (int t = 0; t < nslab; ++t) qi += slab[(int64_t)t * ld + i];
    q[i] = qi;
    if (i < n) {
      const double l = sf2 - qi + sn2;
      const double il = 1.0 / l;
      lam[i] = l;
      inv_lam[i] = il;
      ys[i] = y[i] * il;
      v[0] = log(l);
      v[1] = y[i] * y[i] * il;
    } else {
      lam[i] = 1.0;
      inv_lam[i] = 0.0;  // padded rows carry no weight in B = Kmnᵀ Λ⁻¹ Knm
      ys[i] = 0.0;
    }
  }
  block_sum<2>(v, sh);
  if (threadIdx.x == 0) {
    part[(int64_t)blockIdx.x * 2] = v[0];
    part[(int64_t)blockIdx.x * 2 + 1] = v[1];
  }
}
hipError_t launch_fitc_lambda(const double* slab, int64_t ld, int nslab, const double* y, int n,
                              int n_pad, double sf2, double sn2, double* q, double* lam,
                              double* inv_lam, double* ys, double* scal, double* part,
                              hipStream_t s) {
  const int nblk = std::max(1, (n_pad + 255) / 256);
  hipLaunchKernelGGL(fitc_lambda_rows_kernel, dim3(nblk), dim3(256), 0, s, slab, ld, nslab, y, n,
                     n_pad, sf2, sn2, q, lam, inv_lam, ys, part);
  hipLaunchKernelGGL(partials_sum_kernel<2>, dim3(1), dim3(1024), 0, s, part, nblk, scal);
  return hipGetLastError();
}

// r_i = Σ_t slab_t[i] (the Lb row-norm partials), then the LOO terms: d = 1/λ − r/λ²,
// α = (y − g)/λ → μ = y − α/d, σ² = 1/d (K20:231-232); partial sums [Σ crps, Σ logs]
__global__ __launch_bounds__(256) void fitc_loo_rows_kernel(
    const double* __restrict__ y, const double* __restrict__ lam, const double* __restrict__ slab,
    int64_t ld, int nslab, const double* __restrict__ g, int n, int n_pad, double* __restrict__ r,
    double* __restrict__ mu_loo, double* __restrict__ var_loo, double* __restrict__ part) {
  __shared__ double sh[2 * 16];
  double v[2] = {0.0, 0.0};
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n_pad) {
    double ri = 0.0;
#pragma unroll 8
    for (int t = 0; t < nslab; ++t) ri += slab[(int64_t)t * ld + i];
    r[i] = ri;
    if (i < n) {
      const double il = 1.0 / lam[i];
      const double d = il - ri * il * il;   // diag((Q+Λ)⁻¹), Woodbury
      const double a = (y[i] - g[i]) * il;  // ((Q+Λ)⁻¹ y)_i
      const double m = y[i] - a / d;        // K20:231
      const double c = 1.0 / d;             // K20:232
      mu_loo[i] = m;
      var_loo[i] = c;
      v[0] = crps_term(m, c, y[i]);
      v[1] = logs_term(m, c, y[i]);
    }
  }
  block_sum<2>(v, sh);
  if (threadIdx.x == 0) {
    part[(int64_t)blockIdx.x * 2] = v[0];
    part[(int64_t)blockIdx.x * 2 + 1] = v[1];
  }
}
hipError_t launch_fitc_loo(const double* y, const double* lam, const double* slab, int64_t ld,
                           int nslab, const double* g, int n, int n_pad, double* r,
                           double* mu_loo, double* var_loo, double* sums, double* part,
                           hipStream_t s) {
  const int nblk = std::max(1, (n_pad + 255) / 256);
  hipLaunchKernelGGL(fitc_loo_rows_kernel, dim3(nblk), dim3(256), 0, s, y, lam, slab, ld, nslab, g,
                     n, n_pad, r, mu_loo, var_loo, part);
  hipLaunchKernelGGL(partials_sum_kernel<2>, dim3(1), dim3(1024), 0, s, part, nblk, sums);
  return hipGetLastError();
}

// --------------------------------------------------------------------- small
__global__ __launch_bounds__(1024) void dot_kernel(const double* __restrict__ a,
                                                   const double* __restrict__ b, int n,
                                                   double* __restrict__ out) {
  __shared__ double sh[16];
  double v[1] = {0.0};
  for (int i = threadIdx.x; i < n; i += blockDim.x) v[0] += b ? a[i] * b[i] : a[i];
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) out[0] = v[0];
}
hipError_t launch_dot(const double* a, const double* b, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(1024), 0, s, a, b, n, out);
  return hipGetLastError();
}

// dst (rows_pad × cols_pad, ldd) = src (rows × cols, lds) zero-padded; identity on
// the padded diagonal when pad_identity (used to embed a user SPD matrix)
__global__ __launch_bounds__(256) void pad_copy_kernel(const double* __restrict__ src, int64_t lds,
                                                       double* __restrict__ dst, int64_t ldd, int rows,
                                                       int cols, int rows_pad, int cols_pad,
                                                       int pad_identity) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)rows_pad * cols_pad) return;
  const int i = (int)(e / cols_pad), j = (int)(e - (int64_t)i * cols_pad);
  double v;
  if (i < rows && j < cols) v = src[(int64_t)i * lds + j];
  else v = (pad_identity && i == j) ? 1.0 : 0.0;
  dst[(int64_t)i * ldd + j] = v;
}
hipError_t launch_pad_copy(const double* src, int64_t lds, double* dst, int64_t ldd, int rows,
                           int cols, int rows_pad, int cols_pad, int pad_identity, hipStream_t s) {
  const int64_t tot = (int64_t)rows_pad * cols_pad;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(pad_copy_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src, lds,
                     dst, ldd, rows, cols, rows_pad, cols_pad, pad_identity);
  return hipGetLastError();
}

// in-process all-reduce (api.hip allreduce_sum, local group): out[i] = Σ_q src[q][i] in rank order
// from 0.0 — the same sum, in the same order, as the group's host path
__global__ __launch_bounds__(256) void local_sum_kernel(LocalSumPtrs sp, int n, int64_t count,
                                                        double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  double v = 0.0;
  for (int q = 0; q < n; ++q) v += sp.p[q][i];
  out[i] = v;
}
hipError_t launch_local_sum(const LocalSumPtrs& sp, int n, int64_t count, double* out, hipStream_t s) {
  if (n < 1 || n > kLocalSumMax) return hipErrorInvalidValue;
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(local_sum_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, sp, n,
                     count, out);
  return hipGetLastError();
}

hipError_t launch_trmv_lower(const double* L, int64_t ldl, const double* x, double* y, int n_pad,
                             int trans, hipStream_t s) {
  if (!trans) return launch_gemv_lower(L, ldl, x, y, n_pad, s);
  return hipErrorInvalidValue;  // transposed form goes through launch_colred (needs a slab)
}

}  // namespace gps
