// EXPERIMENT BASELINE (not in the library): the round-1 register-blocked leaf (v3), kept for
// the same-box A/B in tools/diag_bench.cpp.  The library's leaf is the v4 MFMA kernel in
// csrc/kernels_potrf.hip (51 -> 36 us per 128 block, profiles/r2_leaf_v4_diag.txt).
#include "gps_internal.h"

namespace gps {
namespace leafv3 {

constexpr int NB = 128;
constexpr int LTS = 132;

__device__ __forceinline__ void lds_read4(const double* p, double (&v)[4]) {
  const double2 a = *reinterpret_cast<const double2*>(p);
  const double2 b = *reinterpret_cast<const double2*>(p + 2);
  v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}

// ---------------------------------------------------------------------------
// the 528 lower 4×4 blocks are packed column-major into 10 waves, every
// block column inside ONE wave (wave w owns columns [kColStart[w], kColStart[w+1])).
//
//   factor, step jb (one barrier):
//     a. every lane with bc >= jb applies the rank-4 update with L column jb-1
//        (published in CB before the previous barrier);
//     b. the wave owning column jb broadcasts A_jj with v_readlane and ALL its lanes
//        factor it redundantly (Cholesky with one rsqrt per pivot, then D⁻¹), so the
//        panel lanes have D⁻¹ in registers: L_rj = A_rj D⁻ᵀ, published to CB, plus
//        P_rj = L_rj D⁻¹ (kept in LDS for the inverse).  No LDS round trip and no
//        barrier between pivot and panel, which is where the 32-barrier v1 spent
//        most of its time (pivot wave issue-starved, then a second barrier).
//   invert (no barriers): with R = I, for k ascending, R_r,c -= P_r,k R_k,c
//     (column c of L⁻¹ only needs column c of R, which lives in one wave), and
//     finally X = L⁻¹ = D⁻¹ R block row by block row.
// ---------------------------------------------------------------------------
constexpr int V3_WAVES = 10;
__constant__ int kColStart[V3_WAVES + 1] = {0, 2, 4, 6, 8, 10, 13, 16, 20, 27, 32};

__device__ __forceinline__ int wave_of_col(int c) {
  return c < 10 ? (c >> 1) : c < 13 ? 5 : c < 16 ? 6 : c < 20 ? 7 : c < 27 ? 8 : 9;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void wave_lds_fence() {
  // LDS instructions of one wave execute in order; this only stops the compiler
  // from moving LDS accesses across the publish/consume point.
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(64 * V3_WAVES) void potrf_diag_v3_kernel(
    const double* __restrict__ A, int64_t lda, double* __restrict__ Linv, int64_t ldl,
    double* __restrict__ Lout, int64_t ldlo, double* __restrict__ logdiag, int* info, int base,
    int nreal) {
  __shared__ __attribute__((aligned(16))) double PT[NB * LTS];     // PT[col][row] = P[row][col]
  __shared__ __attribute__((aligned(16))) double CB[2 * 4 * NB];   // L column panel [buf][k][row]
  __shared__ __attribute__((aligned(16))) double DI[32 * 16];      // D_b⁻¹ (row-major)
  __shared__ __attribute__((aligned(16))) double DG[NB];           // L_ii
  __shared__ __attribute__((aligned(16))) double XR[V3_WAVES * 7 * 16];  // per-wave published R_k,c

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int cs = kColStart[w], ce = kColStart[w + 1];
  // lane -> (br, bc) inside the wave's columns
  int bc = cs, off = lane;
  while (bc < ce && off >= 32 - bc) {
    off -= 32 - bc;
    ++bc;
  }
  const bool active = bc < ce;
  const int br = active ? bc + off : 0;
  if (!active) bc = 0;
  const int r0 = br * 4, c0 = bc * 4;

  double a[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (active) {
      const double2* src = reinterpret_cast<const double2*>(A + (int64_t)(r0 + r) * lda + c0);
      const double2 u = src[0], v = src[1];
      a[r][0] = u.x; a[r][1] = u.y; a[r][2] = v.x; a[r][3] = v.y;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) a[r][c] = 0.0;
    }
  }

  // ======================= factorisation =======================
  for (int jb = 0; jb < 32; ++jb) {
    const bool mine = w == wave_of_col(jb);  // wave-uniform
    if (mine) __builtin_amdgcn_s_setprio(2);
    if (jb > 0 && active && bc >= jb) {  // a. rank-4 update, L column jb-1
      const double* cb = CB + ((jb - 1) & 1) * 4 * NB;
      double lr[4][4], lc[4][4];  // [k][i]
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lds_read4(&cb[k * NB + r0], lr[k]);
        lds_read4(&cb[k * NB + c0], lc[k]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double s = a[r][c];
#pragma unroll
          for (int k = 0; k < 4; ++k) s = fma(-lr[k][r], lc[k][c], s);
          a[r][c] = s;
        }
    }
    if (mine) {  // b. pivot (redundantly in every lane of this wave) + panel
      int ljj = 0;
      for (int c = cs; c < jb; ++c) ljj += 32 - c;
      ljj = __builtin_amdgcn_readfirstlane(ljj);
      double l[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) l[r][c] = readlane_f64(a[r][c], ljj);
      double is[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double d = l[j][j];  // d <= 0 or NaN leaves L_jj = d*rsqrt(d) NaN: checked after the loop
        is[j] = rsqrt(d);
        l[j][j] = d * is[j];
#pragma unroll
        for (int r = j + 1; r < 4; ++r) l[r][j] *= is[j];
#pragma unroll
        for (int r = j + 1; r < 4; ++r)
#pragma unroll
          for (int c = j + 1; c <= r; ++c) l[r][c] = fma(-l[r][j], l[c][j], l[r][c]);
      }
      // D⁻¹ (lower): x_cc = 1/L_cc, x_rc = -(1/L_rr) Σ_{c<=k<r} L_rk x_kc
      double x[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r < c) {
            x[r][c] = 0.0;
          } else if (r == c) {
            x[r][c] = is[r];
          } else {
            double t = 0.0;
#pragma unroll
            for (int k = c; k < r; ++k) t = fma(l[r][k], x[k][c], t);
            x[r][c] = -t * is[r];
          }
        }
      double* cb = CB + (jb & 1) * 4 * NB;
      if (active && bc == jb && br > jb) {  // panel: L_rj = A_rj D⁻ᵀ, kept in a[][]
        double L[4][4];                     // L[r][c] = Σ_{k<=c} a[r][k] x[c][k]
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k <= c; ++k) s = fma(a[r][k], x[c][k], s);
            L[r][c] = s;
          }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          *reinterpret_cast<double2*>(&cb[c * NB + r0]) = make_double2(L[0][c], L[1][c]);
          *reinterpret_cast<double2*>(&cb[c * NB + r0 + 2]) = make_double2(L[2][c], L[3][c]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) a[r][c] = L[r][c];
      }
      if (lane == ljj) {  // the diagonal block's own lane keeps L_jj (D⁻¹ is rebuilt after the loop)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) a[r][c] = c <= r ? l[r][c] : 0.0;
      }
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
  }
  // ---- off the per-step critical path: D⁻¹ and L_jj of every diagonal block (in parallel)
  if (active && br == bc) {
    // first non-positive pivot (torch.potrf's leading-minor index): a bad pivot makes its
    // L_ii NaN and poisons every later one, so the minimum flagged index is the first
    int bad = 0;
#pragma unroll
    for (int r = 3; r >= 0; --r)
      if (!(a[r][r] > 0.0) && r0 + r < nreal) bad = r0 + r + 1;
    if (bad) atomicMin(info, base + bad);
    double x[4][4];  // x = L_jj⁻¹ (lower): x_cc = 1/L_cc, x_rc = -(1/L_rr) Σ_{c<=k<r} L_rk x_kc
    double is[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) is[r] = 1.0 / a[r][r];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r < c) {
          x[r][c] = 0.0;
        } else if (r == c) {
          x[r][c] = is[r];
        } else {
          double t = 0.0;
#pragma unroll
          for (int k = c; k < r; ++k) t = fma(a[r][k], x[k][c], t);
          x[r][c] = -t * is[r];
        }
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      DG[r0 + r] = a[r][r];
      *reinterpret_cast<double2*>(&DI[br * 16 + r * 4]) = make_double2(x[r][0], x[r][1]);
      *reinterpret_cast<double2*>(&DI[br * 16 + r * 4 + 2]) = make_double2(x[r][2], x[r][3]);
    }
  }
  if (Lout && active) {  // L (diagonal blocks hold zeros above their diagonal)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double2* dst = reinterpret_cast<double2*>(Lout + (int64_t)(r0 + r) * ldlo + c0);
      dst[0] = make_double2(a[r][0], a[r][1]);
      dst[1] = make_double2(a[r][2], a[r][3]);
    }
  }
  __syncthreads();
  if (active && br > bc) {  // P_rb = L_rb D_b⁻¹ for the inverse: P[r][c] = Σ_{k>=c} L[r][k] x[k][c]
    double di[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lds_read4(&DI[bc * 16 + r * 4], di[r]);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int k = c; k < 4; ++k) s = fma(a[r][k], di[k][c], s);
        p[r] = s;
      }
      *reinterpret_cast<double2*>(&PT[(c0 + c) * LTS + r0]) = make_double2(p[0], p[1]);
      *reinterpret_cast<double2*>(&PT[(c0 + c) * LTS + r0 + 2]) = make_double2(p[2], p[3]);
    }
  }
  __syncthreads();
  if (tid < NB) logdiag[tid] = log(DG[tid]);
  if (Lout) {  // zero blocks strictly above the block diagonal
    for (int e = tid; e < NB * 32; e += 64 * V3_WAVES) {
      const int r = e >> 5, zb = e & 31;
      if (zb > (r >> 2)) {
        double2* dst = reinterpret_cast<double2*>(Lout + (int64_t)r * ldlo + zb * 4);
        dst[0] = make_double2(0.0, 0.0);
        dst[1] = make_double2(0.0, 0.0);
      }
    }
  }

  // ======================= X = L⁻¹ (per wave, no barriers) =======================
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) a[r][c] = (active && br == bc && r == c) ? 1.0 : 0.0;
  double* xr = XR + w * 7 * 16;
  for (int k = cs; k < 31; ++k) {
    if (active && br == k) {  // publish R_k,c (final: every update from rows < k applied)
      double* dst = xr + (bc - cs) * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        *reinterpret_cast<double2*>(&dst[r * 4]) = make_double2(a[r][0], a[r][1]);
        *reinterpret_cast<double2*>(&dst[r * 4 + 2]) = make_double2(a[r][2], a[r][3]);
      }
    }
    wave_lds_fence();
    if (active && br > k && bc <= k) {  // R_r,c -= P_r,k R_k,c
      double p[4][4], rk[4][4];          // p[i][r] = P[r0+r][4k+i]; rk[i][c] = R_k,c[i][c]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lds_read4(&PT[(4 * k + i) * LTS + r0], p[i]);
        lds_read4(&xr[(bc - cs) * 16 + i * 4], rk[i]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double s = a[r][c];
#pragma unroll
          for (int i = 0; i < 4; ++i) s = fma(-p[i][r], rk[i][c], s);
          a[r][c] = s;
        }
    }
    wave_lds_fence();
  }
  if (active) {  // X_r,c = D_r⁻¹ R_r,c
    double di[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lds_read4(&DI[br * 16 + r * 4], di[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k <= r; ++k) s = fma(di[r][k], a[k][c], s);
        v[c] = s;
      }
      double2* dst = reinterpret_cast<double2*>(Linv + (int64_t)(r0 + r) * ldl + c0);
      dst[0] = make_double2(v[0], v[1]);
      dst[1] = make_double2(v[2], v[3]);
    }
  }
  for (int e = tid; e < NB * 32; e += 64 * V3_WAVES) {  // zeros above the block diagonal
    const int r = e >> 5, zb = e & 31;
    if (zb > (r >> 2)) {
      double2* dst = reinterpret_cast<double2*>(Linv + (int64_t)r * ldl + zb * 4);
      dst[0] = make_double2(0.0, 0.0);
      dst[1] = make_double2(0.0, 0.0);
    }
  }
}

hipError_t launch_potrf_leaf_v3(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                                int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                                hipStream_t s) {
  if ((lda & 1) || (ldl & 1) || (Lout && (ldlo & 1))) return hipErrorInvalidValue;
  hipLaunchKernelGGL(potrf_diag_v3_kernel, dim3(1), dim3(64 * V3_WAVES), 0, s, A, lda, Linv, ldl,
                     Lout, ldlo, logdiag, info, base, nreal);
  return hipGetLastError();
}

}  // namespace leafv3
}  // namespace gps
