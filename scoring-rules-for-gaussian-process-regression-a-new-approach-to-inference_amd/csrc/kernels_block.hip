// 4-fold block-LOO objectives: DSS (KF:487-543 full GP, K20:523-587
// FITC; dss KF:103-108) and KC = per-fold CRPS of the block-LOO predictive (K20:655-720).
// For fold f with P_f = (A⁻¹)_ff (full GP) or ((Q+Λ)⁻¹)_ff (FITC):
//   m_f = y_f − P_f⁻¹α_f, C_f = P_f⁻¹  (the scripts' chol_solve(I, k_f)·k_inv_y[f])
// P_f is factored by the same recursive potrf_inv as the main matrix; this file holds the
// O(b) per-fold terms, the assembly of ∂obj/∂P_f into the block-diagonal Gblk used by the
// gradient (M = −A⁻¹ Gblk A⁻¹ − ½(vαᵀ + αvᵀ)), and two small helpers.
#include "gps_internal.h"
#include "gpscore.h"

namespace gps {

// One workgroup: m = y − r, c (= diag P⁻¹) → out[0] += Σ crps terms / b (KC), and for the
// gradient gm = ∂(fold-mean crps)/∂m, gc = ∂/∂c (erf-based CDF as in KF:65).
__global__ __launch_bounds__(256) void fold_terms_kernel(const double* __restrict__ y,
                                                         const double* __restrict__ r,
                                                         const double* __restrict__ c, int b,
                                                         double* __restrict__ gm,
                                                         double* __restrict__ gc,
                                                         double* __restrict__ out) {
  __shared__ double sh[16];
  double v[1] = {0.0};
  for (int i = threadIdx.x; i < b; i += 256) {
    const double s = sqrt(c[i]), res = r[i];  // y − m = r
    const double z = res / s;
    const double cdf = 0.5 * (1.0 + erf(z * 0.70710678118654752440));
    const double pdf = 0.39894228040143267794 * exp(-0.5 * z * z);
    v[0] += s * (z * (2.0 * cdf - 1.0) + 2.0 * pdf - 0.56418958354775628695);
    if (gm) {
      gm[i] = (1.0 - 2.0 * cdf) / b;
      gc[i] = (2.0 * pdf - 0.56418958354775628695) / (2.0 * s * b);
    }
  }
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) out[0] = v[0] / b;
}

hipError_t launch_fold_terms(const double* y, const double* r, const double* c, int b, double* gm,
                             double* gc, double* out, hipStream_t s) {
  hipLaunchKernelGGL(fold_terms_kernel, dim3(1), dim3(256), 0, s, y, r, c, b, gm, gc, out);
  return hipGetLastError();
}

// G_f (b×b, written at G with leading dimension ldg) =
//   c0·PI + c1·r rᵀ + c2·½(w rᵀ + r wᵀ) + c3·H      (PI = P⁻¹ full, H = P⁻¹diag(gc)P⁻¹)
// and g[i] = gr·r_i + gw·w_i (the ∂obj/∂α_f entries)
__global__ __launch_bounds__(256) void fold_grad_kernel(const double* __restrict__ PI, int64_t ldp,
                                                        const double* __restrict__ H, int64_t ldh,
                                                        const double* __restrict__ r,
                                                        const double* __restrict__ w, int b,
                                                        double c0, double c1, double c2, double c3,
                                                        double gr, double gw,
                                                        double* __restrict__ G, int64_t ldg,
                                                        double* __restrict__ g) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)b * b) return;
  const int i = (int)(e / b), j = (int)(e - (int64_t)i * b);
  double v = c0 * PI[(int64_t)i * ldp + j] + c1 * r[i] * r[j];
  if (c2 != 0.0) v += c2 * 0.5 * (w[i] * r[j] + r[i] * w[j]);
  if (c3 != 0.0) v += c3 * H[(int64_t)i * ldh + j];
  G[(int64_t)i * ldg + j] = v;
  if (j == 0) g[i] = gr * r[i] + (gw != 0.0 ? gw * w[i] : 0.0);
}

hipError_t launch_fold_grad(const double* PI, int64_t ldp, const double* H, int64_t ldh,
                            const double* r, const double* w, int b, double c0, double c1,
                            double c2, double c3, double gr, double gw, double* G, int64_t ldg,
                            double* g, hipStream_t s) {
  const int64_t tot = (int64_t)b * b;
  hipLaunchKernelGGL(fold_grad_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, PI,
                     ldp, H, ldh, r, w, b, c0, c1, c2, c3, gr, gw, G, ldg, g);
  return hipGetLastError();
}

// ---- FITC block-LOO in low rank (round 5): C_f = Λ_f + W Wᵀ with W = K_f L_{−f}⁻ᵀ (b × m) is
// never formed; every fold quantity comes from products with W (api.hip fitc_lr_folds).

// one wave per row i < rows: at[i] = Σ_k A[i][k]·t[k] (t != null), ab[i] = Σ_k A[i][k]·B[i][k]
// (B != null; B = A gives the row norms).  Lane order fixed: bitwise reproducible.
__global__ __launch_bounds__(256) void row_dots_kernel(const double* __restrict__ A, int64_t lda,
                                                       const double* __restrict__ B, int64_t ldb,
                                                       const double* __restrict__ t, int rows,
                                                       int cols, double* __restrict__ at,
                                                       double* __restrict__ ab) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const double* a = A + (int64_t)row * lda;
  const double* bb = B ? B + (int64_t)row * ldb : nullptr;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 2 * lane; k < cols; k += 128) {
    const double2 av = *reinterpret_cast<const double2*>(a + k);
    if (t) {
      const double2 tv = *reinterpret_cast<const double2*>(t + k);
      s1 = fma(av.x, tv.x, s1);
      s1 = fma(av.y, tv.y, s1);
    }
    if (bb) {
      const double2 bv = *reinterpret_cast<const double2*>(bb + k);
      s2 = fma(av.x, bv.x, s2);
      s2 = fma(av.y, bv.y, s2);
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    if (t) at[row] = s1;
    if (bb) ab[row] = s2;
  }
}

hipError_t launch_row_dots(const double* A, int64_t lda, const double* B, int64_t ldb,
                           const double* t, int rows, int cols, double* at, double* ab,
                           hipStream_t s) {
  if ((cols & 1) || (lda & 1) || (B && (ldb & 1)) || rows <= 0) return rows == 0 ? hipSuccess : hipErrorInvalidValue;
  hipLaunchKernelGGL(row_dots_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, A, lda, B,
                     ldb, t, rows, cols, at, ab);
  return hipGetLastError();
}

// the per-row fold vectors, i < bp (rows b..bp-1 get 0):
//   mode 0: o1 = r = λx + at, o2 = c = λ + ab                      (x = α_f)
//   mode 1: o1 = w = λx + at                                       (x = gm)
//   mode 2 (KC):  o1 = diag G_f = w∘r − (λ²gc + 2λ·gc·(c − λ) + q),  o2 = g_f = −w
//   mode 3 (DSS): o1 = diag G_f = −½(c + r²),                         o2 = g_f = r
__global__ __launch_bounds__(256) void lr_fold_vec_kernel(int mode, int b, int bp,
                                                          const double* __restrict__ lam,
                                                          const double* __restrict__ x,
                                                          const double* __restrict__ at,
                                                          const double* __restrict__ ab,
                                                          const double* __restrict__ r,
                                                          const double* __restrict__ c,
                                                          const double* __restrict__ w,
                                                          const double* __restrict__ gc,
                                                          const double* __restrict__ q,
                                                          double* __restrict__ o1,
                                                          double* __restrict__ o2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= bp) return;
  if (i >= b) {
    o1[i] = 0.0;
    if (o2) o2[i] = 0.0;
    return;
  }
  const double l = lam[i];
  switch (mode) {
    case 0: o1[i] = fma(l, x[i], at[i]); o2[i] = l + ab[i]; break;
    case 1: o1[i] = fma(l, x[i], at[i]); break;
    case 2: {
      const double g = gc[i];
      o1[i] = w[i] * r[i] - (l * l * g + 2.0 * l * g * (c[i] - l) + q[i]);
      o2[i] = -w[i];
      break;
    }
    default: o1[i] = -0.5 * (c[i] + r[i] * r[i]); o2[i] = r[i]; break;
  }
}

hipError_t launch_lr_fold_vec(int mode, int b, int bp, const double* lam, const double* x,
                              const double* at, const double* ab, const double* r, const double* c,
                              const double* w, const double* gc, const double* q, double* o1,
                              double* o2, hipStream_t s) {
  if (bp <= 0) return hipSuccess;
  hipLaunchKernelGGL(lr_fold_vec_kernel, dim3((unsigned)((bp + 255) / 256)), dim3(256), 0, s, mode,
                     b, bp, lam, x, at, ab, r, c, w, gc, q, o1, o2);
  return hipGetLastError();
}

// out[i][j] = rs_i·c0·(X[i][j] + λ_i·Y[i][j]) + c1·u1_i·v1_j + c2·u2_i·v2_j for i < rows (rs, the
// rank-one terms optional), 0 for rows ≤ i < rows_pad; j < cols
__global__ __launch_bounds__(256) void lr_combine_kernel(const double* __restrict__ X, int64_t ldx,
                                                         const double* __restrict__ Y, int64_t ldy,
                                                         const double* __restrict__ lam,
                                                         const double* __restrict__ rs, double c0,
                                                         const double* __restrict__ u1,
                                                         const double* __restrict__ v1, double c1,
                                                         const double* __restrict__ u2,
                                                         const double* __restrict__ v2, double c2,
                                                         int rows, int rows_pad, int cols,
                                                         double* __restrict__ out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)rows_pad * cols) return;
  const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
  double v = 0.0;
  if (i < rows) {
    v = c0 * fma(lam[i], Y[(int64_t)i * ldy + j], X[(int64_t)i * ldx + j]);
    if (rs) v *= rs[i];
    if (u1) v = fma(c1 * u1[i], v1[j], v);
    if (u2) v = fma(c2 * u2[i], v2[j], v);
  }
  out[(int64_t)i * ldo + j] = v;
}

hipError_t launch_lr_combine(const double* X, int64_t ldx, const double* Y, int64_t ldy,
                             const double* lam, const double* rs, double c0, const double* u1,
                             const double* v1, double c1, const double* u2, const double* v2,
                             double c2, int rows, int rows_pad, int cols, double* out, int64_t ldo,
                             hipStream_t s) {
  const int64_t tot = (int64_t)rows_pad * cols;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(lr_combine_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, ldx,
                     Y, ldy, lam, rs, c0, u1, v1, c1, u2, v2, c2, rows, rows_pad, cols, out, ldo);
  return hipGetLastError();
}

// P[i][i] += vals[i] for i < nreal; P[i][i] = 1 for nreal <= i < npad (diag(P, I) embedding)
__global__ __launch_bounds__(256) void add_diag_kernel(double* __restrict__ P, int64_t ld,
                                                       const double* __restrict__ vals, int nreal,
                                                       int npad) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= npad) return;
  double* p = P + (int64_t)i * ld + i;
  *p = i < nreal ? *p + vals[i] : 1.0;
}

hipError_t launch_add_diag(double* P, int64_t ld, const double* vals, int nreal, int npad,
                           hipStream_t s) {
  hipLaunchKernelGGL(add_diag_kernel, dim3((npad + 255) / 256), dim3(256), 0, s, P, ld, vals, nreal,
                     npad);
  return hipGetLastError();
}

// FITC block-LOO covariance (round 5, api.hip fitc_fold_cov): dst[e] = base[e] (+ base2[e]) +
// sgn·Σ_{g ≠ skip} slab_g[e], the slabs in ascending order (fixed: bitwise reproducible); e < len
__global__ __launch_bounds__(256) void fold_sum_kernel(const double* __restrict__ slab, int64_t stride,
                                                       int nslab, int skip, const double* base,
                                                       const double* base2, double sgn,
                                                       double* dst, int64_t len) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= len) return;
  double v = base ? base[e] : 0.0;
  if (base2) v += base2[e];
  for (int g = 0; g < nslab; ++g)
    if (g != skip) v = fma(sgn, slab[g * stride + e], v);
  dst[e] = v;
}

hipError_t launch_fold_sum(const double* slab, int64_t stride, int nslab, int skip, const double* base,
                           const double* base2, double sgn, double* dst, int64_t len, hipStream_t s) {
  hipLaunchKernelGGL(fold_sum_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, slab,
                     stride, nslab, skip, base, base2, sgn, dst, len);
  return hipGetLastError();
}

// *out = Σ_{i<m} ldf[i] − Σ_{i<m} ldb[i] − ½Σ_{i<b} log lam[i] = −½log|C_f| of the fold covariance
// C_f = Λ_f + K_f B_{−f}⁻¹K_fᵀ (log|C_f| = Σ log λ_f + log|B| − log|B_{−f}|; ld* = log L_ii of
// the two factors) — the P-sign convention of blockloo_folds' ½log|P_f| slot.  One workgroup.
__global__ __launch_bounds__(256) void fold_logdet_kernel(const double* __restrict__ ldf,
                                                          const double* __restrict__ ldb, int m,
                                                          const double* __restrict__ lam, int b,
                                                          double* __restrict__ out) {
  __shared__ double sh[16];
  double v[1] = {0.0};
  for (int i = threadIdx.x; i < m; i += 256) v[0] += ldf[i] - ldb[i];
  for (int i = threadIdx.x; i < b; i += 256) v[0] -= 0.5 * log(lam[i]);
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) *out = v[0];
}

hipError_t launch_fold_logdet(const double* ldf, const double* ldb, int m, const double* lam, int b,
                              double* out, hipStream_t s) {
  hipLaunchKernelGGL(fold_logdet_kernel, dim3(1), dim3(256), 0, s, ldf, ldb, m, lam, b, out);
  return hipGetLastError();
}

// M[i][:] *= scale[i] for i < rows (cols even)
__global__ __launch_bounds__(256) void row_scale_kernel(double* __restrict__ M, int64_t ld, int rows,
                                                        int cols, const double* __restrict__ scale) {
  const int64_t e = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (e >= (int64_t)rows * cols) return;
  const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
  double2* p = reinterpret_cast<double2*>(M + (int64_t)i * ld + j);
  const double sc = scale[i];
  double2 v = *p;
  v.x *= sc;
  v.y *= sc;
  *p = v;
}

hipError_t launch_row_scale(double* M, int64_t ld, int rows, int cols, const double* scale,
                            hipStream_t s) {
  if (cols & 1) return hipErrorInvalidValue;
  const int64_t pairs = (int64_t)rows * cols / 2;
  hipLaunchKernelGGL(row_scale_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s, M, ld,
                     rows, cols, scale);
  return hipGetLastError();
}

// out[i] = a[i]·b[i] (i < n)
__global__ __launch_bounds__(256) void vec_mul_kernel(const double* __restrict__ a,
                                                      const double* __restrict__ b, int n,
                                                      double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

hipError_t launch_vec_mul(const double* a, const double* b, int n, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(vec_mul_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

// ------------------------------------------- FITC block-LOO gradient (K20:587, K20:720)
// Whitened (round 4, api.hip gps_fitc_blockloo): with Ũ = Λ⁻¹K Lb⁻ᵀ, F̃ = Gblk Ũ, S̃ = ŨᵀF̃,
//   M_ii = −G_ii/λ_i² + 2 F̃_i·Ũ_i/λ_i − (ŨS̃)_i·Ũ_i − v_iα_i,
// the row scale of G_K's V Lm⁻¹ term sc = −2M_ii, and the left factor of its Lb⁻¹ term
// Y = −2Λ⁻¹F̃ + 2ŨS̃ (written over Y, which may alias US: each element is read, then written, by
// the same lane).  One wave per row (HBM-bound: one pass over F̃, ŨS̃, Ũ); pad rows get zeros.
__global__ __launch_bounds__(256) void blk_mdiag_kernel(
    const double* __restrict__ F, int64_t ldf, const double* US, int64_t ldus,
    const double* __restrict__ U, int64_t ldu, int m_pad, const double* __restrict__ gd,
    const double* __restrict__ lam, const double* __restrict__ v,
    const double* __restrict__ alpha, int n, int n_pad, double* __restrict__ md,
    double* __restrict__ sc, double* Y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_pad) return;
  double* y = Y + (int64_t)i * ldy;
  if (i >= n) {
    if (lane == 0) md[i] = sc[i] = 0.0;
    for (int j = 2 * lane; j < m_pad; j += 128) *reinterpret_cast<double2*>(y + j) = double2{0.0, 0.0};
    return;
  }
  const double* f = F + (int64_t)i * ldf;
  const double* us = US + (int64_t)i * ldus;
  const double* u = U + (int64_t)i * ldu;
  const double il = 1.0 / lam[i];
  double p = 0.0, q = 0.0;
  for (int j = 2 * lane; j < m_pad; j += 128) {
    const double2 uv = *reinterpret_cast<const double2*>(u + j);
    const double2 fv = *reinterpret_cast<const double2*>(f + j);
    const double2 sv = *reinterpret_cast<const double2*>(us + j);
    p = fma(fv.x, uv.x, p);
    p = fma(fv.y, uv.y, p);
    q = fma(sv.x, uv.x, q);
    q = fma(sv.y, uv.y, q);
    *reinterpret_cast<double2*>(y + j) =
        double2{fma(-2.0 * il, fv.x, 2.0 * sv.x), fma(-2.0 * il, fv.y, 2.0 * sv.y)};
  }
  p = wave_sum(p);
  q = wave_sum(q);
  if (lane == 0) {
    const double mi = -gd[i] * il * il + 2.0 * p * il - q - v[i] * alpha[i];
    md[i] = mi;
    sc[i] = -2.0 * mi;
  }
}

hipError_t launch_blk_mdiag(const double* F, int64_t ldf, const double* US, int64_t ldus,
                            const double* U, int64_t ldu, int m_pad, const double* gd,
                            const double* lam, const double* v, const double* alpha, int n,
                            int n_pad, double* md, double* sc, double* Y, int64_t ldy,
                            hipStream_t s) {
  if ((ldf & 1) || (ldus & 1) || (ldu & 1) || (ldy & 1) || (m_pad & 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(blk_mdiag_kernel, dim3((n_pad + 3) / 4), dim3(256), 0, s, F, ldf, US, ldus, U,
                     ldu, m_pad, gd, lam, v, alpha, n, n_pad, md, sc, Y, ldy);
  return hipGetLastError();
}

// ------------------------------------------------------------ energy score (KF:70-101)
// The square root C^½ comes from the coupled Newton–Schulz iteration in the MFMA GEMM
// (api.hip es_fold); these are its elementwise steps and the distance / reduction stages.

// Y (bp×bp) = diag(scale·C_b, pad·I): C's real b×b block (ldc) scaled, or scale·I when C is
// null; the padded diagonal gets `pad` (1 keeps the padded block a fixed point of the
// iteration, 0 for its derivative block)
__global__ __launch_bounds__(256) void ns_init_kernel(const double* __restrict__ C, int64_t ldc,
                                                      int b, int bp, double scale, double pad,
                                                      double* __restrict__ Y) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)bp * bp) return;
  const int i = (int)(e / bp), j = (int)(e - (int64_t)i * bp);
  double v;
  if (i < b && j < b) v = C ? scale * C[(int64_t)i * ldc + j] : (i == j ? scale : 0.0);
  else v = i == j ? pad : 0.0;
  Y[e] = v;
}

hipError_t launch_ns_init(const double* C, int64_t ldc, int b, int bp, double scale, double pad,
                          double* Y, hipStream_t s) {
  const int64_t tot = (int64_t)bp * bp;
  hipLaunchKernelGGL(ns_init_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, C, ldc, b,
                     bp, scale, pad, Y);
  return hipGetLastError();
}

// M_ii += c (i < n)
__global__ __launch_bounds__(256) void diag_add_const_kernel(double* __restrict__ M, int64_t ld,
                                                             int n, double c) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) M[(int64_t)i * ld + i] += c;
}

hipError_t launch_diag_add_const(double* M, int64_t ld, int n, double c, hipStream_t s) {
  hipLaunchKernelGGL(diag_add_const_kernel, dim3((n + 255) / 256), dim3(256), 0, s, M, ld, n, c);
  return hipGetLastError();
}

// M ← ½(M + Mᵀ) in place (n×n; one thread per pair i > j)
__global__ __launch_bounds__(256) void sym_avg_kernel(double* __restrict__ M, int64_t ld, int n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
  if (j >= i) return;
  double* a = M + (int64_t)i * ld + j;
  double* b = M + (int64_t)j * ld + i;
  const double v = 0.5 * (*a + *b);
  *a = v;
  *b = v;
}

hipError_t launch_sym_avg(double* M, int64_t ld, int n, hipStream_t s) {
  const int64_t tot = (int64_t)n * n;
  hipLaunchKernelGGL(sym_avg_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, M, ld, n);
  return hipGetLastError();
}

// dst[j] = scale·src[j] (j < b), 0 (b <= j < bp)
__global__ __launch_bounds__(256) void scaled_row_kernel(const double* __restrict__ src, int b,
                                                         int bp, double scale,
                                                         double* __restrict__ dst) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < bp) dst[j] = j < b ? scale * src[j] : 0.0;
}

hipError_t launch_scaled_row(const double* src, int b, int bp, double scale, double* dst,
                             hipStream_t s) {
  hipLaunchKernelGGL(scaled_row_kernel, dim3((bp + 255) / 256), dim3(256), 0, s, src, b, bp, scale,
                     dst);
  return hipGetLastError();
}

// C[i][j] += s[i]·Z[i][j]
__global__ __launch_bounds__(256) void row_axpy_kernel(double* __restrict__ C, int64_t ldc,
                                                       const double* __restrict__ Z, int64_t ldz,
                                                       const double* __restrict__ sv, int rows,
                                                       int cols) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)rows * cols) return;
  const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
  double* c = C + (int64_t)i * ldc + j;
  *c = fma(sv[i], Z[(int64_t)i * ldz + j], *c);
}

hipError_t launch_row_axpy(double* C, int64_t ldc, const double* Z, int64_t ldz, const double* sv,
                           int rows, int cols, hipStream_t s) {
  const int64_t tot = (int64_t)rows * cols;
  hipLaunchKernelGGL(row_axpy_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, C, ldc, Z,
                     ldz, sv, rows, cols);
  return hipGetLastError();
}

// out = Σ_ij (T_ij − δ_ij)² (n×n, one workgroup, fixed order): the iteration's convergence
// check when no spectral bounds are known (gps_energy_score)
__global__ __launch_bounds__(1024) void ns_resid_kernel(const double* __restrict__ T, int64_t ld,
                                                        int n, double* __restrict__ out) {
  __shared__ double sh[16];
  double v[1] = {0.0};
  const int64_t tot = (int64_t)n * n;
  for (int64_t e = threadIdx.x; e < tot; e += 1024) {
    const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
    const double t = T[(int64_t)i * ld + j] - (i == j ? 1.0 : 0.0);
    v[0] = fma(t, t, v[0]);
  }
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) out[0] = v[0];
}

hipError_t launch_ns_resid(const double* T, int64_t ld, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(ns_resid_kernel, dim3(1), dim3(1024), 0, s, T, ld, n, out);
  return hipGetLastError();
}

// D[i][j] = ‖z_i − ẑ_j‖ for i < S, j <= S (rows of length bp, zero past b): the direct
// differences ES forms (KF:86-88, 94-96).  16×16 pairs per workgroup, k staged through LDS
// (rows padded to 65 doubles: the 16 ẑ rows a wave reads land on distinct banks).
__global__ __launch_bounds__(256) void es_dist_kernel(const double* __restrict__ Z,
                                                      const double* __restrict__ Zh, int64_t ld,
                                                      int S, int bp, double* __restrict__ D,
                                                      int64_t ldd) {
  __shared__ double za[16][65], zb[16][65];
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
  double acc = 0.0;
  for (int k0 = 0; k0 < bp; k0 += 64) {
    for (int e = threadIdx.x; e < 16 * 64; e += 256) {
      const int r = e >> 6, k = e & 63;
      za[r][k] = i0 + r < S ? Z[(int64_t)(i0 + r) * ld + k0 + k] : 0.0;
      zb[r][k] = j0 + r <= S ? Zh[(int64_t)(j0 + r) * ld + k0 + k] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < 64; ++k) {
      const double t = za[ti][k] - zb[tj][k];
      acc = fma(t, t, acc);
    }
    __syncthreads();
  }
  const int i = i0 + ti, j = j0 + tj;
  if (i < S && j <= S) D[(int64_t)i * ldd + j] = sqrt(acc);
}

hipError_t launch_es_dist(const double* Z, const double* Zh, int64_t ld, int S, int bp, double* D,
                          int64_t ldd, hipStream_t s) {
  if (bp % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(es_dist_kernel, dim3((S + 1 + 15) / 16, (S + 15) / 16), dim3(256), 0, s, Z, Zh,
                     ld, S, bp, D, ldd);
  return hipGetLastError();
}

// ES = (1/S)Σ_i D_iS^β − Σ_{i,j<S} D_ij^β / (2S(S−1)) → out[0] (KF:91, 97-100).  With grad, D
// is overwritten by W = ∂ES/∂D ∘ D⁻¹ = coef_j·β·D^(β−2) (zero-padded to Sp×Sp) and its row /
// column sums go to rs / cs.  One workgroup, fixed order.
__global__ __launch_bounds__(1024) void es_reduce_kernel(double* __restrict__ D, int64_t ldd, int S,
                                                         int Sp, double beta, int grad,
                                                         double* __restrict__ rs,
                                                         double* __restrict__ cs,
                                                         double* __restrict__ out) {
  __shared__ double sh[2 * 16];
  const double cz = 1.0 / ((double)S * (S - 1)), cy = 1.0 / S;
  const bool b1 = beta == 1.0;
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < Sp; i += 1024) {
    double* row = D + (int64_t)i * ldd;
    double rsum = 0.0;
    if (i < S) {
      for (int j = 0; j <= S; ++j) {
        const double dd = row[j];
        const double pb = b1 ? dd : pow(dd, beta);
        if (j < S) v[0] += pb;
        else v[1] += pb;
        if (grad) {
          const double wv = (j < S ? -0.5 * cz : cy) * (b1 ? 1.0 / dd : beta * pb / (dd * dd));
          row[j] = wv;
          rsum += wv;
        }
      }
    }
    if (grad) {
      for (int j = i < S ? S + 1 : 0; j < Sp; ++j) row[j] = 0.0;
      rs[i] = rsum;
    }
  }
  block_sum<2>(v, sh);  // ends with a barrier: W is complete for the column sums
  if (threadIdx.x == 0) out[0] = cy * v[1] - 0.5 * cz * v[0];
  if (!grad) return;
  for (int j = threadIdx.x; j < Sp; j += 1024) {
    double c = 0.0;
    for (int i = 0; i < S; ++i) c += D[(int64_t)i * ldd + j];
    cs[j] = c;
  }
}

hipError_t launch_es_reduce(double* D, int64_t ldd, int S, int Sp, double beta, int grad,
                            double* rs, double* cs, double* out, hipStream_t s) {
  if (S < 2 || Sp < S + 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(es_reduce_kernel, dim3(1), dim3(1024), 0, s, D, ldd, S, Sp, beta, grad, rs, cs,
                     out);
  return hipGetLastError();
}

}  // namespace gps
