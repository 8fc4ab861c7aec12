// FP64 MFMA GEMM for gfx950 — the one genuinely dense contraction of the GP hot path.
//
// Every O(n^3) / O(n m^2) step of the build reduces to this kernel:
//   * Cholesky trailing update  A22 -= L21 L21ᵀ        (SYRK, lower tiles only)
//   * TRSM as a product with the diagonal inverse       L21 = A21 L11⁻ᵀ
//   * triangular inverse off-diagonal blocks            L⁻¹21 = -L22⁻¹ (L21 L11⁻¹)
//   * predictive TRMM with fused column reductions      colsum((L⁻¹K_f*)²), (L⁻¹K_f*)ᵀβ
//   * FITC: ‖Lm⁻¹k_i‖² / ‖Lb⁻¹k_i‖² row reductions, B = Kmnᵀ Λ⁻¹ Knm (split-K SYRK)
// (reference: chol_solve KF:25-29, half-logdet KF:332, cal_mean_and_cov KF:121-126,
//  Q KF:32-39, spgp_cal_mean_and_cov K20:76-83 — all LAPACK/BLAS on the CPU there).
//
// Geometry: 128×128 output tile per 256-thread workgroup (4 waves, each a 64×64
// sub-tile = 4×4 blocks of v_mfma_f64_16x16x4_f64), K staged through LDS in
// 16-deep slices, double-buffered (global→register prefetch of slice k+1 while
// slice k is multiplied).  LDS images are k-major [k][128 + 16]: a fragment read
// (16 consecutive doubles per k row, 4 k rows per wave instruction) then hits
// all 64 banks without conflict (row stride ≡ 32 dwords mod 64).
//
// f64 MFMA operand map (cdna_hip_programming.md §3): lane l supplies
// A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15]; accumulator register r of
// lane l is C[row = (l>>4) + 4r][col = l&15].
//
// Triangular operands are handled by clipping the K range per output tile at
// 128-granularity (the diagonal tiles of a triangular factor are stored with
// explicit zeros above the diagonal), so no multiply touches a tile that is
// structurally zero.  Workgroup ids are remapped so that the tiles one XCD
// runs are contiguous in tile order (shared A rows stay in that XCD's L2).
#include "gps_internal.h"

namespace gps {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 16, LS = 144;
constexpr int STAGE = 2 * BK * LS;  // doubles per buffer (A image + B image)

constexpr int GROUP_M = 8;

// logical tile id -> (ti, tj).  Lower-triangular enumeration for SYRK outputs;
// otherwise a grouped raster (GROUP_M tile rows at a time, column-major inside
// the group) so the tiles resident together share A and B panels in L2.  For
// triangular operands the tiles with the longest K range are issued first.
__device__ __forceinline__ void tile_of(const GemmParams& p, int t, int& ti, int& tj) {
  if (p.lower_out) {
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    ti = r;
    tj = t - r * (r + 1) / 2;
    return;
  }
  const int per_group = GROUP_M * p.tiles_n;
  const int g = t / per_group;
  const int first = g * GROUP_M;
  const int gm = min(GROUP_M, p.tiles_m - first);
  const int tt = t - g * per_group;
  ti = first + tt % gm;
  tj = tt / gm;
  if (p.tri == TRI_K_LE_I) ti = p.tiles_m - 1 - ti;
  else if (p.tri == TRI_K_LE_J) tj = p.tiles_n - 1 - tj;
}

// bijective XCD-contiguous remap: blocks b, b+8, b+16, ... (one XCD under the
// observed round-robin dispatch) get consecutive logical tile ids.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <int ALAY, int BLAY, int EPI>
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) double smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  int ti, tj;
  tile_of(p, xcd_remap(blockIdx.x, gridDim.x), ti, tj);
  const int row0 = ti * BM, col0 = tj * BN;

  int kb = 0, ke = p.K;
  switch (p.tri) {
    case TRI_K_LE_I: ke = min(ke, row0 + BM); break;
    case TRI_K_LE_J: ke = min(ke, col0 + BN); break;
    case TRI_K_GE_J: kb = col0; break;
    case TRI_K_GE_I: kb = row0; break;
    default: break;
  }
  if (p.ksplit > 1) {
    const int nk = ke > kb ? (ke - kb) / BK : 0;
    const int s = blockIdx.y, q = nk / p.ksplit, r = nk % p.ksplit;
    const int s0 = s * q + min(s, r), s1 = s0 + q + (s < r ? 1 : 0);
    ke = kb + s1 * BK;
    kb = kb + s0 * BK;
  }
  const int nk = ke > kb ? (ke - kb) / BK : 0;

  // ---- global -> register staging (8 doubles of A and 8 of B per thread) ----
  double2 ra[4], rb[4];
  auto load_tile = [&](int k0) {
    if constexpr (ALAY == LAY_T) {  // A stored [k][i]
      const int k = tid >> 4, i = (tid & 15) * 8;
      const double2* src = reinterpret_cast<const double2*>(p.A + (int64_t)(k0 + k) * p.lda + row0 + i);
#pragma unroll
      for (int q = 0; q < 4; ++q) ra[q] = src[q];
      if (p.kscale) {
        const double sc = p.kscale[k0 + k];
#pragma unroll
        for (int q = 0; q < 4; ++q) { ra[q].x *= sc; ra[q].y *= sc; }
      }
    } else {  // A stored [i][k]
      const int i = tid >> 1, k = (tid & 1) * 8;
      const double2* src = reinterpret_cast<const double2*>(p.A + (int64_t)(row0 + i) * p.lda + k0 + k);
#pragma unroll
      for (int q = 0; q < 4; ++q) ra[q] = src[q];
      if (p.kscale) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ra[q].x *= p.kscale[k0 + k + 2 * q];
          ra[q].y *= p.kscale[k0 + k + 2 * q + 1];
        }
      }
    }
    if constexpr (BLAY == LAY_N) {  // B stored [k][j]
      const int k = tid >> 4, j = (tid & 15) * 8;
      const double2* src = reinterpret_cast<const double2*>(p.B + (int64_t)(k0 + k) * p.ldb + col0 + j);
#pragma unroll
      for (int q = 0; q < 4; ++q) rb[q] = src[q];
    } else {  // B stored [j][k]
      const int j = tid >> 1, k = (tid & 1) * 8;
      const double2* src = reinterpret_cast<const double2*>(p.B + (int64_t)(col0 + j) * p.ldb + k0 + k);
#pragma unroll
      for (int q = 0; q < 4; ++q) rb[q] = src[q];
    }
  };
  auto store_tile = [&](int buf) {
    double* As = smem + buf * STAGE;
    double* Bs = As + BK * LS;
    if constexpr (ALAY == LAY_T) {
      const int k = tid >> 4, i = (tid & 15) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<double2*>(&As[k * LS + i + 2 * q]) = ra[q];
    } else {
      const int i = tid >> 1, k = (tid & 1) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        As[(k + 2 * q) * LS + i] = ra[q].x;
        As[(k + 2 * q + 1) * LS + i] = ra[q].y;
      }
    }
    if constexpr (BLAY == LAY_N) {
      const int k = tid >> 4, j = (tid & 15) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<double2*>(&Bs[k * LS + j + 2 * q]) = rb[q];
    } else {
      const int j = tid >> 1, k = (tid & 1) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Bs[(k + 2 * q) * LS + j] = rb[q].x;
        Bs[(k + 2 * q + 1) * LS + j] = rb[q].y;
      }
    }
  };

  d4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (d4){0.0, 0.0, 0.0, 0.0};

  auto compute = [&](int buf) {
    const double* As = smem + buf * STAGE;
    const double* Bs = As + BK * LS;
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int krow = (kk * 4 + (lane >> 4)) * LS + (lane & 15);
      double a[4], b[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = As[krow + wr * 64 + mi * 16];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b[ni] = Bs[krow + wc * 64 + ni * 16];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  if (nk > 0) {
    load_tile(kb);
    store_tile(0);
    __syncthreads();
    // steady state: prefetch slice it+1 into registers, multiply slice it, then
    // park the prefetched slice in the other LDS buffer (no branches in the body)
    for (int it = 0; it < nk - 1; ++it) {
      load_tile(kb + (it + 1) * BK);
      compute(it & 1);
      store_tile((it + 1) & 1);
      __syncthreads();
    }
    compute((nk - 1) & 1);
  }

  const int lrow = lane >> 4, lcol = lane & 15;
  if constexpr (EPI == EPI_STORE) {
    double* Cb = p.C + (int64_t)blockIdx.y * p.c_kslice_stride;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wr * 64 + mi * 16 + lrow + 4 * r;
        double* crow = Cb + (int64_t)row * p.ldc + col0 + wc * 64 + lcol;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          double v = p.alpha * acc[mi][ni][r];
          if (p.beta != 0.0) v = fma(p.beta, crow[ni * 16], v);
          crow[ni * 16] = v;
        }
      }
  } else if constexpr (EPI == EPI_ROWSQ) {
    // out0[tj][row] = sum over this tile's 128 columns of (alpha*acc)^2
    double* red = smem;  // [2 (wc)][128 rows]
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) s = fma(acc[mi][ni][r], acc[mi][ni][r], s);
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        if (lcol == 0) red[wc * 128 + wr * 64 + mi * 16 + lrow + 4 * r] = s;
      }
    __syncthreads();
    if (tid < 128)
      p.out0[(int64_t)tj * p.ld_out + row0 + tid] = p.alpha * p.alpha * (red[tid] + red[128 + tid]);
  } else {  // EPI_COLRED: out0[ti][col] = sum_rows w[row]*acc, out1[ti][col] = sum_rows acc^2
    double* red = smem;  // [2 (wr)][2][128]
    __syncthreads();
    double wv[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) wv[mi][r] = p.w[row0 + wr * 64 + mi * 16 + lrow + 4 * r];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1 = fma(acc[mi][ni][r], wv[mi][r], s1);
          s2 = fma(acc[mi][ni][r], acc[mi][ni][r], s2);
        }
      s1 += __shfl_xor(s1, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 16);
      s2 += __shfl_xor(s2, 32);
      if (lrow == 0) {
        red[wr * 256 + wc * 64 + ni * 16 + lcol] = s1;
        red[wr * 256 + 128 + wc * 64 + ni * 16 + lcol] = s2;
      }
    }
    __syncthreads();
    if (tid < 128) {
      p.out0[(int64_t)ti * p.ld_out + col0 + tid] = p.alpha * (red[tid] + red[256 + tid]);
      p.out1[(int64_t)ti * p.ld_out + col0 + tid] =
          p.alpha * p.alpha * (red[128 + tid] + red[384 + tid]);
    }
  }
}

hipError_t launch_gemm(int alay, int blay, int epi, const GemmParams& pin, hipStream_t s) {
  GemmParams p = pin;
  if (p.M % BM || p.N % BN || p.K % BK || p.M <= 0 || p.N <= 0) return hipErrorInvalidValue;
  if ((p.lda & 1) || (p.ldb & 1) || (p.ldc & 1)) return hipErrorInvalidValue;
  if (p.lower_out && p.M != p.N) return hipErrorInvalidValue;
  if (p.ksplit < 1) p.ksplit = 1;
  if (p.ksplit > 1 && (epi != EPI_STORE || p.beta != 0.0)) return hipErrorInvalidValue;
  p.tiles_m = p.M / BM;
  p.tiles_n = p.N / BN;
  const int tiles = p.lower_out ? p.tiles_m * (p.tiles_m + 1) / 2 : p.tiles_m * p.tiles_n;
  dim3 grid(tiles, p.ksplit), block(256);
#define GPS_GEMM_CASE(AL, BL, EP)                                                   \
  if (alay == AL && blay == BL && epi == EP) {                                     \
    hipLaunchKernelGGL((gemm_f64_kernel<AL, BL, EP>), grid, block, 0, s, p);       \
    return hipGetLastError();                                                      \
  }
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_STORE)
  GPS_GEMM_CASE(LAY_N, LAY_N, EPI_STORE)
  GPS_GEMM_CASE(LAY_T, LAY_N, EPI_STORE)
  GPS_GEMM_CASE(LAY_T, LAY_T, EPI_STORE)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_ROWSQ)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_COLRED)
#undef GPS_GEMM_CASE
  return hipErrorInvalidValue;
}

}  // namespace gps
