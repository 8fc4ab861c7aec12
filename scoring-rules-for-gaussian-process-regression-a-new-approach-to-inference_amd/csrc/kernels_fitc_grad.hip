// Analytic FITC gradients — the quantities the reference obtains with autograd
// `.backward()` through its dense n×n FITC bodies at K20:236 (LOO-CRPS), K20:344 (NLML)
// and K20:452 (LOO-LogS), w.r.t. (para_k, para_l, para_noise) AND the inducing inputs
// (trained in the reference, K20:247).  Restated in O(n·m²) (oracle.fast_fitc_grad):
//
//   C = Q + Λ, Q = K Km⁻¹ Kᵀ (K = Knm, Km = K(Z,Z) + 1e-3·I), Λ = diag(K_ff − Q) + σ²I
//   ∂obj = tr(M ∂C),  M = a·C⁻¹ − ½(vαᵀ + αvᵀ) − C⁻¹ diag(h) C⁻¹
//   tr(M ∂C) = Σ G_K ∘ ∂K + Σ G_Km ∘ ∂Km + Σ_i M_ii (∂K_ii + ∂σ²)
//   G_K  = (s1 ∘ U + s2 ∘ U P) Lb⁻¹ + s3 ∘ (V Lm⁻¹) − v cᵀ − α ŵᵀ      (row scales s1..s3)
//   G_Km = a(B⁻¹ − Km⁻¹) + Lb⁻ᵀ P Lb⁻¹ + Lm⁻ᵀ(Vᵀdiag(M_ii)V)Lm⁻¹ + ½(ŵcᵀ + cŵᵀ)
// whitened (round 4): U = K Lb⁻ᵀ, V = K Lm⁻ᵀ, P = Uᵀdiag(h/λ²)U — no explicit Km⁻¹ / B⁻¹ in the
// n×m products (K B⁻¹ = U Lb⁻¹, K Km⁻¹ = V Lm⁻¹, K N = U P Lb⁻¹)
// The m×m and n×m products run in the MFMA GEMM (api.hip); this file holds the per-row
// terms and the contraction of G with ∂K/∂θ and ∂K/∂Z, which recomputes K_ij and the
// scaled differences from the features instead of storing d+2 derivative matrices.
#include "gps_internal.h"
#include "gpscore.h"

namespace gps {

// ------------------------------------------------------------------ per-row terms
// α = (y − g)/λ, d = 1/λ − r/λ²  (g = K c, r = k_iB⁻¹k_iᵀ from the forward)
// NLML: v = ½α, h = 0.  LOO: u = −g_μ/d, h = (g_μα − g_c)/d², ulam = u/λ (v needs C⁻¹u).
// hl2 = h/λ² (the per-k scale of the S2 = Kᵀdiag(h/λ²)K SYRK).
__global__ __launch_bounds__(256) void fitc_grad_terms_kernel(
    const double* __restrict__ y, const double* __restrict__ lam, const double* __restrict__ r,
    const double* __restrict__ g, int n, int n_pad, int obj, double n_total,
    double* __restrict__ alpha, double* __restrict__ dinv, double* __restrict__ v,
    double* __restrict__ ulam, double* __restrict__ h, double* __restrict__ hl2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_pad) return;
  if (i >= n) {
    alpha[i] = dinv[i] = v[i] = ulam[i] = h[i] = hl2[i] = 0.0;
    return;
  }
  const double l = lam[i], il = 1.0 / l;
  const double a = (y[i] - g[i]) * il;
  const double d = il - r[i] * il * il;
  alpha[i] = a;
  dinv[i] = d;
  if (obj == GPS_OBJ_NLML) {
    v[i] = 0.5 * a;
    ulam[i] = h[i] = hl2[i] = 0.0;
    return;
  }
  const double c = 1.0 / d, res = a / d;  // LOO variance, y − μ_loo
  double gm, gc;
  if (obj == GPS_OBJ_LOO_CRPS) {  // K20 crps (≡ KF:60-68)
    const double s = sqrt(c), z = res / s;
    const double cdf = 0.5 * (1.0 + erf(z * 0.70710678118654752440));
    const double pdf = 0.39894228040143267794 * exp(-0.5 * z * z);
    gm = 1.0 - 2.0 * cdf;
    gc = (2.0 * pdf - 0.56418958354775628695) / (2.0 * s);
  } else {  // logs (≡ KF:52-57); K20:446's variance equals 1/d algebraically
    gm = -res / c;
    gc = 0.5 / c - res * res / (2.0 * c * c);
  }
  gm /= n_total;
  gc /= n_total;
  const double u = -gm / d, hh = (gm * a - gc) / (d * d);
  v[i] = 0.0;
  ulam[i] = u * il;
  h[i] = hh;
  hl2[i] = hh * il * il;
}

hipError_t launch_fitc_grad_terms(const double* y, const double* lam, const double* r,
                                  const double* g, int n, int n_pad, int obj, double n_total,
                                  double* alpha, double* dinv, double* v, double* ulam, double* h,
                                  double* hl2, hipStream_t s) {
  hipLaunchKernelGGL(fitc_grad_terms_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, s, y, lam, r,
                     g, n, n_pad, obj, n_total, alpha, dinv, v, ulam, h, hl2);
  return hipGetLastError();
}

// v = ulam − z/λ  (v = C⁻¹u by Woodbury, z = U Uᵀ(u/λ)); lam NULL: v = ulam − z
__global__ __launch_bounds__(256) void fitc_grad_v_kernel(const double* __restrict__ ulam,
                                                          const double* __restrict__ z,
                                                          const double* __restrict__ lam, int n,
                                                          double* __restrict__ v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = ulam[i] - (lam ? z[i] / lam[i] : z[i]);
}

hipError_t launch_fitc_grad_v(const double* ulam, const double* z, const double* lam, int n,
                              double* v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fitc_grad_v_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ulam, z, lam, n, v);
  return hipGetLastError();
}

// One wave per row: q_i = Σ_j (U P)_ij U_ij = k_i N k_iᵀ (skipped when KN is null: h = 0), then
//   M_ii = a·d_i − v_iα_i − (h_i/λ_i² − 2h_i r_i/λ_i³ + q_i/λ_i²)
//   s1 = 2(a/λ − h/λ²), s2 = 2/λ, s3 = −2 M_ii  (row scales of G_K); pad rows: all 0.
__global__ __launch_bounds__(256) void fitc_grad_mdiag_kernel(
    const double* __restrict__ KN, int64_t ldkn, const double* __restrict__ K, int64_t ldk,
    int m_pad, const double* __restrict__ lam, const double* __restrict__ r,
    const double* __restrict__ dinv, const double* __restrict__ alpha,
    const double* __restrict__ v, const double* __restrict__ h, double a, int n, int n_pad,
    double* __restrict__ mdiag, double* __restrict__ s1, double* __restrict__ s2,
    double* __restrict__ s3) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_pad) return;
  if (i >= n) {
    if (lane == 0) mdiag[i] = s1[i] = s2[i] = s3[i] = 0.0;
    return;
  }
  double q = 0.0;
  if (KN) {
    const double* kn = KN + (int64_t)i * ldkn;
    const double* kr = K + (int64_t)i * ldk;
    for (int j = 2 * lane; j < m_pad; j += 128) {
      const double2 x = *reinterpret_cast<const double2*>(kn + j);
      const double2 k = *reinterpret_cast<const double2*>(kr + j);
      q = fma(x.x, k.x, q);
      q = fma(x.y, k.y, q);
    }
    q = wave_sum(q);
  }
  if (lane == 0) {
    const double il = 1.0 / lam[i], hi = h ? h[i] : 0.0;
    const double md =
        a * dinv[i] - v[i] * alpha[i] - (hi * il * il - 2.0 * hi * r[i] * il * il * il + q * il * il);
    mdiag[i] = md;
    s1[i] = 2.0 * (a * il - hi * il * il);
    s2[i] = 2.0 * il;
    s3[i] = -2.0 * md;
  }
}

hipError_t launch_fitc_grad_mdiag(const double* KN, int64_t ldkn, const double* K, int64_t ldk,
                                  int m_pad, const double* lam, const double* r, const double* dinv,
                                  const double* alpha, const double* v, const double* h, double a,
                                  int n, int n_pad, double* mdiag, double* s1, double* s2,
                                  double* s3, hipStream_t s) {
  hipLaunchKernelGGL(fitc_grad_mdiag_kernel, dim3((n_pad + 3) / 4), dim3(256), 0, s, KN, ldkn, K,
                     ldk, m_pad, lam, r, dinv, alpha, v, h, a, n, n_pad, mdiag, s1, s2, s3);
  return hipGetLastError();
}

// Y = diag(s1)·U + diag(s2)·UP over rows × cols (UP null: the s2 term is absent); Y may alias UP
// (the whitened G_K's left factor, api.hip gps_fitc_grad)
__global__ __launch_bounds__(256) void fitc_grad_y_kernel(const double* __restrict__ U,
                                                          const double* UP, int64_t ld,
                                                          const double* __restrict__ s1,
                                                          const double* __restrict__ s2, int rows,
                                                          int cols, double* Y) {
  const int64_t e = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (e >= (int64_t)rows * cols) return;
  const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
  const int64_t o = (int64_t)i * ld + j;
  const double2 u = *reinterpret_cast<const double2*>(U + o);
  const double a = s1[i];
  double2 y = {a * u.x, a * u.y};
  if (UP) {
    const double2 w = *reinterpret_cast<const double2*>(UP + o);
    const double b = s2[i];
    y.x = fma(b, w.x, y.x);
    y.y = fma(b, w.y, y.y);
  }
  *reinterpret_cast<double2*>(Y + o) = y;
}

hipError_t launch_fitc_grad_y(const double* U, const double* UP, int64_t ld, const double* s1,
                              const double* s2, int rows, int cols, double* Y, hipStream_t s) {
  if ((cols & 1) || (ld & 1) || rows <= 0) return hipErrorInvalidValue;
  const int64_t pairs = (int64_t)rows * cols / 2;
  hipLaunchKernelGGL(fitc_grad_y_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s, U,
                     UP, ld, s1, s2, rows, cols, Y);
  return hipGetLastError();
}

// ---------------------------------------------------------------- contraction
// Grid (column blocks of 64, row chunks of p.rchunk, dimension passes of 16).  Thread
// (rg, cj) owns column j = 64·bx + cj and rows rg, rg+4, … of the chunk.  Per element
//   G_ij = Σ_t coef_t·(rs_t ? rs_t[i] : 1)·R_t[i][j] + Σ_q pc_q·p_q[i]·q_q[j]
//   Δ_k = (xr_ik − xc_jk)/ℓ_k, K_ij = sf2·exp(−½ Σ_k Δ_k²), GK = G_ij·K_ij
//   acc: Σ GK, Σ GK Δ_k² (this pass's dims), and per column Σ_i GK Δ_k (→ Z gradient)
constexpr int FG_COLS = 64;
constexpr int FG_DP = 16;
constexpr int FG_U = 4;  // rows per thread per batch (loads issued together)

template <int D>
__global__ __launch_bounds__(256) void fitc_grad_contract_kernel(FitcContractParams p) {
  extern __shared__ double xs[];  // [64 cols][d] scaled column features (D == 0 path)
  __shared__ double sh[(1 + FG_DP) * 16];
  __shared__ double zsh[4][FG_COLS][FG_DP + 1];
  __shared__ double2 etab[64];
  const int d = D > 0 ? D : p.d;
  const int d0 = blockIdx.z * FG_DP;
  const int cj = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * FG_COLS + cj;
  const int r0 = blockIdx.y * p.rchunk, r1 = min(p.nr, r0 + p.rchunk);
  if constexpr (D == 0) {
    for (int e = threadIdx.x; e < FG_COLS * d; e += 256) {
      const int q = e / d, k = e - q * d, jj = blockIdx.x * FG_COLS + q;
      xs[e] = jj < p.nc ? p.xc[(int64_t)jj * d + k] * p.inv_ell[k] : 0.0;
    }
  }
  exp_tab_stage(etab);
  __syncthreads();
  double xj[D > 0 ? D : 1];
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) xj[k] = j < p.nc ? p.xc[(int64_t)j * D + k] * p.inv_ell[k] : 0.0;
  }
  double acc[1 + FG_DP], zacc[FG_DP];
#pragma unroll
  for (int q = 0; q < 1 + FG_DP; ++q) acc[q] = 0.0;
#pragma unroll
  for (int q = 0; q < FG_DP; ++q) zacc[q] = 0.0;
  if (j < p.nc) {
    double qj[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) qj[q] = p.pc[q] != 0.0 ? p.qv[q][j] : 0.0;
    // rows in batches of FG_U per thread: every R[t] load (and the wave-uniform rs[t][i]
    // scalar loads) of the batch is issued before the first element's arithmetic, so
    // FG_U·nt HBM reads are in flight per wave instead of one (the one-row loop waited
    // out a full HBM latency per element).  Rows are still accumulated in ascending order,
    // so the sums are bitwise those of the one-row loop.
    for (int i0 = r0 + rg; i0 < r1; i0 += 4 * FG_U) {
      double Rv[FG_U][4], rsv[FG_U][4];
#pragma unroll
      for (int u = 0; u < FG_U; ++u) {
        const int iu = __builtin_amdgcn_readfirstlane(i0 + 4 * u);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          Rv[u][t] = 0.0;
          rsv[u][t] = 1.0;
          if (iu < r1 && t < p.nt) {
            Rv[u][t] = p.R[t][(int64_t)iu * p.ldr[t] + j];
            if (p.rs[t]) rsv[u][t] = p.rs[t][iu];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < FG_U; ++u) {
        const int iu = __builtin_amdgcn_readfirstlane(i0 + 4 * u);
        if (iu >= r1) break;
        const double* xri = p.xr + (int64_t)iu * d;
        double r2 = 0.0;
        if constexpr (D > 0) {
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const double tk = xri[k] * p.inv_ell[k] - xj[k];
            r2 = fma(tk, tk, r2);
          }
        } else {
          for (int k = 0; k < d; ++k) {
            const double tk = xri[k] * p.inv_ell[k] - xs[cj * d + k];
            r2 = fma(tk, tk, r2);
          }
        }
        const double Kij = p.sf2 * exp_neg(-0.5 * r2, etab);
        double G = 0.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < p.nt) {
            const double sc = p.rs[t] ? p.coef[t] * rsv[u][t] : p.coef[t];
            G = fma(sc, Rv[u][t], G);
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (p.pc[q] != 0.0) G = fma(p.pc[q] * p.pv[q][iu], qj[q], G);
        const double gk = G * Kij;
        acc[0] += gk;
#pragma unroll
        for (int q = 0; q < FG_DP; ++q) {
          if (D > 0 ? q < D : d0 + q < d) {
            const double tq = D > 0 ? xri[q] * p.inv_ell[q] - xj[q]
                                    : xri[d0 + q] * p.inv_ell[d0 + q] - xs[cj * d + d0 + q];
            acc[1 + q] = fma(gk, tq * tq, acc[1 + q]);
            zacc[q] = fma(gk, tq, zacc[q]);
          }
        }
      }
    }
  }
  // per-column Z partials: fixed-order sum over the 4 row groups
#pragma unroll
  for (int q = 0; q < FG_DP; ++q) zsh[rg][cj][q] = zacc[q];
  block_sum<1 + FG_DP>(acc, sh);  // contains __syncthreads
  const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {
    double* o = p.slab + (int64_t)blk * (1 + FG_DP);
#pragma unroll
    for (int q = 0; q < 1 + FG_DP; ++q) o[q] = acc[q];
  }
  // zslab[pass][chunk][j][q]
  for (int e = threadIdx.x; e < FG_COLS * FG_DP; e += 256) {
    const int c = e / FG_DP, q = e - c * FG_DP;
    const int jj = blockIdx.x * FG_COLS + c;
    if (jj < p.nc_pad) {
      const double z = zsh[0][c][q] + zsh[1][c][q] + zsh[2][c][q] + zsh[3][c][q];
      p.zslab[(((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * p.nc_pad + jj) * FG_DP + q] = z;
    }
  }
}

// out[pass*(1+DP) + q] = Σ over the blocks of the pass; zout[j*d + d0+q] = Σ over chunks
__global__ __launch_bounds__(256) void fitc_grad_reduce_kernel(const double* __restrict__ slab,
                                                               int blocks_per_pass,
                                                               double* __restrict__ out) {
  __shared__ double sh[16];
  const int pass = blockIdx.x / (1 + FG_DP), q = blockIdx.x % (1 + FG_DP);
  double v[1] = {0.0};
  for (int t = threadIdx.x; t < blocks_per_pass; t += 256)
    v[0] += slab[((int64_t)pass * blocks_per_pass + t) * (1 + FG_DP) + q];
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) out[pass * (1 + FG_DP) + q] = v[0];
}

__global__ __launch_bounds__(256) void fitc_gradz_reduce_kernel(const double* __restrict__ zslab,
                                                                int chunks, int nc, int nc_pad,
                                                                int d, double* __restrict__ zout) {
  const int e = blockIdx.x * 256 + threadIdx.x;  // e = j*d + k
  if (e >= nc * d) return;
  const int j = e / d, k = e - j * d, pass = k / FG_DP, q = k % FG_DP;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c)
    s += zslab[(((int64_t)pass * chunks + c) * nc_pad + j) * FG_DP + q];
  zout[e] = s;
}

int fitc_contract_passes(int d) { return (d + FG_DP - 1) / FG_DP; }

static int fitc_chunk_rows(int nr) {  // <= 256 row chunks, at least 256 rows each
  int c = (nr + 255) / 256;
  c = (c + 63) / 64 * 64;
  return c < 256 ? 256 : c;
}

int64_t fitc_contract_slab_doubles(int nr, int nc_pad, int d) {
  const int64_t chunks = (nr + fitc_chunk_rows(nr) - 1) / fitc_chunk_rows(nr);
  const int64_t cb = (nc_pad + FG_COLS - 1) / FG_COLS, passes = fitc_contract_passes(d);
  return passes * chunks * cb * (1 + FG_DP) + passes * chunks * nc_pad * FG_DP;
}

hipError_t launch_fitc_grad_contract(FitcContractParams p, double* out, double* zout,
                                     hipStream_t s) {
  if (p.d < 1 || p.d > GPS_MAX_D || p.nt > 4 || p.nr <= 0 || p.nc <= 0) return hipErrorInvalidValue;
  p.rchunk = fitc_chunk_rows(p.nr);
  const int chunks = (p.nr + p.rchunk - 1) / p.rchunk;
  const int cb = (p.nc_pad + FG_COLS - 1) / FG_COLS, passes = fitc_contract_passes(p.d);
  double* slab = p.slab;
  p.zslab = slab + (int64_t)passes * chunks * cb * (1 + FG_DP);
  const dim3 grid(cb, chunks, passes), block(256);
  const size_t lds = (size_t)FG_COLS * p.d * sizeof(double);
  switch (p.d) {
    case 1: hipLaunchKernelGGL(fitc_grad_contract_kernel<1>, grid, block, 0, s, p); break;
    case 8: hipLaunchKernelGGL(fitc_grad_contract_kernel<8>, grid, block, 0, s, p); break;
    case 16: hipLaunchKernelGGL(fitc_grad_contract_kernel<16>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(fitc_grad_contract_kernel<0>, grid, block, lds, s, p); break;
  }
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(fitc_grad_reduce_kernel, dim3(passes * (1 + FG_DP)), dim3(256), 0, s, slab,
                     cb * chunks, out);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(fitc_gradz_reduce_kernel, dim3((p.nc * p.d + 255) / 256), dim3(256), 0, s,
                     p.zslab, chunks, p.nc, p.nc_pad, p.d, zout);
  return hipGetLastError();
}

}  // namespace gps
