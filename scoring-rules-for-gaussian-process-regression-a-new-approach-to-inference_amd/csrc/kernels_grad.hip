// Analytic hyper-parameter gradients of the full-GP objectives — the quantities the
// reference obtains with autograd `.backward()` at KF:252 (LOO-CRPS), KF:339 (NLML)
// and KF:428 (LOO-LogS), then uses for its SGD step (KF:254-260).
//
// Every objective gradient has the form ∂obj/∂θ = Σ_ij M_ij ∂A_ij/∂θ with A = K + σ²I:
//   NLML:  M = ½(A⁻¹ − ααᵀ)
//   LOO:   M = −½(vαᵀ + αvᵀ) − A⁻¹ diag(c̃) A⁻¹,  u = −g_μ/d, c̃ = (g_μα − g_c)/d²,
//          v = A⁻¹u, with (g_μ, g_c) the per-point derivatives of the mean score
//          w.r.t. the LOO mean μ_i = y_i − α_i/d_i and variance c_i = 1/d_i.
// The O(n³) parts (A⁻¹ = L⁻ᵀL⁻¹ and A⁻¹ diag(c̃) A⁻¹) run in the MFMA GEMM; this
// file holds the O(n) per-point terms, the symmetric mirror, and the contraction
// with ∂A/∂θ, which recomputes K_ij and Δ_ij² from X instead of storing d+2
// derivative matrices (one read of M per element: HBM-bound).
#include "gps_internal.h"
#include "gpscore.h"

namespace gps {

// ---------------------------------------------------------------- per-point terms
__global__ __launch_bounds__(256) void loo_grad_terms_kernel(const double* __restrict__ y,
                                                             const double* __restrict__ alpha,
                                                             const double* __restrict__ dinv,
                                                             int n, int n_pad, int obj,
                                                             double* __restrict__ u,
                                                             double* __restrict__ ct) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_pad) return;
  if (i >= n) {
    u[i] = 0.0;
    ct[i] = 0.0;
    return;
  }
  const double d = dinv[i], a = alpha[i];
  const double m = y[i] - a / d, c = 1.0 / d, r = y[i] - m;
  double gm, gc;
  if (obj == GPS_OBJ_LOO_CRPS) {  // KF:60-68: ∂/∂m = 1 − 2Φ(z), ∂/∂c = (2φ(z) − 1/√π)/(2σ)
    const double s = sqrt(c), z = r / s;
    const double cdf = 0.5 * (1.0 + erf(z * 0.70710678118654752440));
    const double pdf = 0.39894228040143267794 * exp(-0.5 * z * z);
    gm = 1.0 - 2.0 * cdf;
    gc = (2.0 * pdf - 0.56418958354775628695) / (2.0 * s);
  } else {  // KF:52-57 LogS: ∂/∂m = −(y−m)/c, ∂/∂c = 1/(2c) − (y−m)²/(2c²)
    gm = -r / c;
    gc = 0.5 / c - r * r / (2.0 * c * c);
  }
  gm /= n;  // the objectives are means over the n points
  gc /= n;
  u[i] = -gm / d;
  ct[i] = (gm * a - gc) / (d * d);
}

hipError_t launch_loo_grad_terms(const double* y, const double* alpha, const double* dinv, int n,
                                 int n_pad, int obj, double* u, double* ct, hipStream_t s) {
  hipLaunchKernelGGL(loo_grad_terms_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, s, y, alpha,
                     dinv, n, n_pad, obj, u, ct);
  return hipGetLastError();
}

// ------------------------------------------------------------ symmetric mirror
// copy the strictly-lower 32-tiles of M into the strictly-upper ones (transposed
// through LDS so both the read and the write are row-coalesced).  The lower-output
// GEMM writes whole tiles of 64 or 128 on and below the diagonal, so every diagonal
// 32-tile is already full; all strictly-lower ones are mirrored.
__global__ __launch_bounds__(256) void sym_mirror_kernel(double* __restrict__ M, int64_t ld,
                                                         int tiles32) {
  __shared__ double t[32][33];
  // blockIdx.x enumerates strictly-lower 32-tiles (r > c) of a tiles32 × tiles32 grid
  const int b = blockIdx.x;
  int r = (int)((sqrt(8.0 * (double)b + 1.0) + 1.0) * 0.5);
  while (r * (r - 1) / 2 > b) --r;
  while ((r + 1) * r / 2 <= b) ++r;
  const int c = b - r * (r - 1) / 2;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 × 8
#pragma unroll
  for (int k = 0; k < 4; ++k)
    t[ty + 8 * k][tx] = M[(int64_t)(r * 32 + ty + 8 * k) * ld + c * 32 + tx];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k)
    M[(int64_t)(c * 32 + ty + 8 * k) * ld + r * 32 + tx] = t[tx][ty + 8 * k];
}

hipError_t launch_sym_mirror(double* M, int64_t ld, int n_pad, hipStream_t s) {
  const int t = n_pad / 32;
  const int64_t blocks = (int64_t)t * (t - 1) / 2;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(sym_mirror_kernel, dim3((unsigned)blocks), dim3(256), 0, s, M, ld, t);
  return hipGetLastError();
}

// ∞-norm of a symmetric n×n block, an upper bound of its spectral radius (the energy score's
// Newton–Schulz scale): one wave per row (coalesced), fixed-order lane sums, then one block
// takes the max (order-free)
__global__ __launch_bounds__(256) void row_abs_sum_kernel(const double* __restrict__ A, int64_t lda,
                                                          int n, double* __restrict__ rowsum) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const double* row = A + (int64_t)r * lda;
  double s = 0.0;
  for (int j = lane; j < n; j += 64) s += fabs(row[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) rowsum[r] = s;
}
__global__ __launch_bounds__(256) void max_kernel(const double* __restrict__ v, int n,
                                                  double* __restrict__ out) {
  __shared__ double red[256];
  double m = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) m = fmax(m, v[i]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}
hipError_t launch_norm_inf(const double* A, int64_t lda, int n, double* rowsum, double* out,
                           hipStream_t s) {
  if (n < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_abs_sum_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, A, lda, n,
                     rowsum);
  hipLaunchKernelGGL(max_kernel, dim3(1), dim3(256), 0, s, rowsum, n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- contraction
// One workgroup per lower 64×64 tile of the REAL n×n region; thread (rg, col) handles
// column col and rows rg, rg+4, …, rg+60.  Per element:
//   m = a0·Ainv_ij + a1·α_iα_j + a2·½(v_iα_j + α_iv_j) + a3·Mx_ij
//   w = 2 off the diagonal (the lower triangle stands for both), 1 on it
//   K_ij = sf2·exp(−½ Σ_k Δ_k²), Δ_k = (x_ik − x_jk)/ℓ_k  (recomputed, as in gram_kernel)
//   acc: [Σ w m K, Σ_{i=j} m, Σ w m K Δ_k² for k in this pass's dims]
// Dimensions beyond DP per pass take extra passes (blockIdx.y), each re-reading M.
constexpr int GT = 64;
constexpr int DP = 16;
constexpr int GU = 4;  // rows per thread per load batch

// D > 0: compile-time feature count (the column's scaled features live in registers);
// D = 0: runtime d <= GPS_MAX_D (features from LDS).  Row features are read from LDS by
// all 64 lanes of a wave at the same address (broadcast, conflict-free).
template <int D>
__global__ __launch_bounds__(256) void grad_contract_kernel(GradParams p) {
  extern __shared__ double xs[];  // [GT rows][d] then [GT cols][d]
  __shared__ double sh[(2 + DP) * 16];
  __shared__ double2 etab[64];
  const int d = D > 0 ? D : p.d;
  const int b = blockIdx.x, pass = blockIdx.y, d0 = pass * DP;
  int ti = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= b) ++ti;
  while (ti * (ti + 1) / 2 > b) --ti;
  const int tj = b - ti * (ti + 1) / 2;
  const int row0 = ti * GT, col0 = tj * GT;
  double* xr = xs;
  double* xc = xs + GT * d;
  for (int e = threadIdx.x; e < GT * d; e += 256) {
    const int q = e / d, k = e - q * d;
    xr[e] = row0 + q < p.n ? p.x[(int64_t)(row0 + q) * d + k] * p.inv_ell[k] : 0.0;
    xc[e] = col0 + q < p.n ? p.x[(int64_t)(col0 + q) * d + k] * p.inv_ell[k] : 0.0;
  }
  exp_tab_stage(etab);
  __syncthreads();
  const int cj = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = col0 + cj;
  double xj[D > 0 ? D : 1];
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) xj[k] = xc[cj * D + k];
  }
  double acc[2 + DP];
#pragma unroll
  for (int q = 0; q < 2 + DP; ++q) acc[q] = 0.0;
  if (j < p.n) {
    const double aj = p.alpha[j], vj = p.v ? p.v[j] : 0.0;
    // rows in batches of GU per thread: the batch's M loads (Ainv, Mx) are all issued before
    // the first element's arithmetic instead of one HBM latency per element; rows are still
    // accumulated in ascending order (bitwise the one-row loop's sums)
    for (int rb = rg; rb < GT; rb += 4 * GU) {
      double ldA[GU], ldX[GU];
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int i = row0 + rb + 4 * u;
        const bool ok = i < p.n && i >= j;
        ldA[u] = ok && p.a0 != 0.0 ? p.Ainv[(int64_t)i * p.ldm + j] : 0.0;
        ldX[u] = ok && p.a3 != 0.0 ? p.Mx[(int64_t)i * p.ldm + j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int rr = rb + 4 * u;
        const int i = row0 + rr;
        if (i >= p.n || i < j) continue;
        double r2 = 0.0;
        if constexpr (D > 0) {
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const double t = xr[rr * D + k] - xj[k];
            r2 = fma(t, t, r2);
          }
        } else {
          for (int k = 0; k < d; ++k) {
            const double t = xr[rr * d + k] - xc[cj * d + k];
            r2 = fma(t, t, r2);
          }
        }
        const double K = p.sf2 * exp_neg(-0.5 * r2, etab);
        const double ai = p.alpha[i];
        double m = p.a1 * ai * aj;
        if (p.a0 != 0.0) m = fma(p.a0, ldA[u], m);
        if (p.a2 != 0.0) m = fma(p.a2, 0.5 * (p.v[i] * aj + ai * vj), m);
        if (p.a3 != 0.0) m = fma(p.a3, ldX[u], m);
        const double w = i == j ? 1.0 : 2.0;
        const double mk = w * m * K;
        acc[0] += mk;
        if (i == j) acc[1] += m;
        if constexpr (D > 0) {  // D <= DP: one pass, d0 == 0
#pragma unroll
          for (int q = 0; q < D; ++q) {
            const double t = xr[rr * D + q] - xj[q];
            acc[2 + q] = fma(mk, t * t, acc[2 + q]);
          }
        } else {
#pragma unroll
          for (int q = 0; q < DP; ++q) {
            if (d0 + q < d) {
              const double t = xr[rr * d + d0 + q] - xc[cj * d + d0 + q];
              acc[2 + q] = fma(mk, t * t, acc[2 + q]);
            }
          }
        }
      }
    }
  }
  block_sum<2 + DP>(acc, sh);
  if (threadIdx.x == 0) {
    double* o = p.slab + ((int64_t)pass * gridDim.x + b) * (2 + DP);
#pragma unroll
    for (int q = 0; q < 2 + DP; ++q) o[q] = acc[q];
  }
}

// out[pass][0..1+DP] = fixed-order sums over the tiles of each pass
__global__ __launch_bounds__(256) void grad_slab_reduce_kernel(const double* __restrict__ slab,
                                                               int tiles, double* __restrict__ out) {
  __shared__ double sh[16];
  const int pass = blockIdx.x / (2 + DP), q = blockIdx.x % (2 + DP);
  double v[1] = {0.0};
  for (int t = threadIdx.x; t < tiles; t += 256)
    v[0] += slab[((int64_t)pass * tiles + t) * (2 + DP) + q];
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) out[pass * (2 + DP) + q] = v[0];
}

int grad_contract_passes(int d) { return (d + DP - 1) / DP; }
int64_t grad_contract_slab_doubles(int n, int d) {
  const int64_t t = (n + GT - 1) / GT;
  return t * (t + 1) / 2 * (2 + DP) * grad_contract_passes(d);
}

hipError_t launch_grad_contract(const GradParams& p, double* out, hipStream_t s) {
  if (p.d < 1 || p.d > GPS_MAX_D) return hipErrorInvalidValue;
  const int t = (p.n + GT - 1) / GT;
  const int tiles = t * (t + 1) / 2, passes = grad_contract_passes(p.d);
  const size_t lds = (size_t)2 * GT * p.d * sizeof(double);
  const dim3 grid(tiles, passes), block(256);
  switch (p.d) {
    case 1: hipLaunchKernelGGL(grad_contract_kernel<1>, grid, block, lds, s, p); break;
    case 8: hipLaunchKernelGGL(grad_contract_kernel<8>, grid, block, lds, s, p); break;
    case 16: hipLaunchKernelGGL(grad_contract_kernel<16>, grid, block, lds, s, p); break;
    default: hipLaunchKernelGGL(grad_contract_kernel<0>, grid, block, lds, s, p); break;
  }
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(grad_slab_reduce_kernel, dim3(passes * (2 + DP)), dim3(256), 0, s, p.slab,
                     tiles, out);
  return hipGetLastError();
}

}  // namespace gps
