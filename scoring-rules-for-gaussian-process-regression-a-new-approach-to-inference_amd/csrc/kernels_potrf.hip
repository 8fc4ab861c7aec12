// Diagonal-block kernel of the blocked Cholesky (replaces LAPACK ?potrf behind
// torch.potrf, KF:26 / KF:332) fused with the block's triangular inverse.
//
// One 640-thread workgroup owns a 128×128 fp64 block held as 4×4 sub-blocks in
// registers; log L_ii (the ½log|A| terms of KF:332) is taken for all 128 pivots in
// parallel after the factorisation.  Details at potrf_diag_v3_kernel.
#include "gps_internal.h"

namespace gps {

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

// ---------------------------------------------------------------------------
// v4: one 256-thread workgroup, the 128 block as 36 lower 16×16 tiles in LDS (row stride 17
// doubles: both the MFMA accumulator-order and operand-order accesses are ~conflict-free),
// 78 KB — small enough to share a CU with one 128-tile GEMM workgroup.  Right-looking over 8
// panels of 16 columns with a lookahead of one panel:
//   phase A (step p)  wave 0 factors panel p (128×16, lane l: rows l, l+64) column by column:
//                     pivot by v_readlane, one rsqrt, multipliers of column j published once
//                     to LDS and read back as broadcasts (the next pivot's by v_readlane);
//                     waves 1-3 meanwhile apply panel p-1 to the tiles of columns ≥ p+1
//                     (v_mfma_f64_16x16x4, 4 per tile), invert L_{p-1,p-1} (16×16, by
//                     substitution) and form T_k = Σ_{j=k}^{p-2} L_{p-1,j} X_{j,k} in registers;
//   phase B (step p)  waves 1-3 apply panel p to column p+1 only (what panel p+1 needs) and
//                     finish X_{p-1,k} = −X_{p-1,p-1} T_k (the accumulators ARE the B operand).
// The inverse X = L⁻¹ (left-looking trtri by block rows) thus trails the factorisation by
// one panel and overwrites L's tiles row by row; L itself goes to Lout from the pivot wave.
// Measured per-panel pivot cost (tools/panel_probe.hip): 3.5k cycles (one row slot) to 5.2k
// (two).  log L_ii and torch.potrf's first non-positive minor come from the pivots.
namespace v4 {
typedef double d4 __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));
constexpr int TS = 17;         // LDS row stride of a tile (doubles)
constexpr int TSZ = 16 * TS;   // one tile slot
constexpr int NT = 36;         // lower tiles of the 8×8 grid
__device__ __forceinline__ constexpr int tix(int i, int j) { return i * (i + 1) / 2 + j; }

__device__ __forceinline__ double rl(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// operand-order element of tile t for k-step kk: (row l & 15, col 4kk + (l >> 4))
__device__ __forceinline__ double opnd(const double* S, int t, int lane, int kk) {
  return S[t * TSZ + (lane & 15) * TS + 4 * kk + (lane >> 4)];
}
// accumulator-order element q: (row 4q + (l >> 4), col l & 15)
__device__ __forceinline__ int acc_off(int t, int lane, int q) {
  return t * TSZ + (4 * q + (lane >> 4)) * TS + (lane & 15);
}
// S_dst −= L_a L_bᵀ (all three tiles in LDS)
__device__ __forceinline__ void tile_update(double* S, int dst, int ta, int tb, int lane) {
  d4 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = S[acc_off(dst, lane, q)];
  double a[4], b[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) { a[kk] = -opnd(S, ta, lane, kk); b[kk] = opnd(S, tb, lane, kk); }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = mfma(a[kk], b[kk], acc);
#pragma unroll
  for (int q = 0; q < 4; ++q) S[acc_off(dst, lane, q)] = acc[q];
}

// two independent updates, all operand loads issued before the MFMAs (tb shared)
__device__ __forceinline__ void tile_update2(double* S, int d0, int a0, int d1, int a1, int tb,
                                             int lane) {
  d4 c0, c1;
  double x0[4], x1[4], b[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) { c0[q] = S[acc_off(d0, lane, q)]; c1[q] = S[acc_off(d1, lane, q)]; }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    x0[kk] = -opnd(S, a0, lane, kk);
    x1[kk] = -opnd(S, a1, lane, kk);
    b[kk] = opnd(S, tb, lane, kk);
  }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) { c0 = mfma(x0[kk], b[kk], c0); c1 = mfma(x1[kk], b[kk], c1); }
#pragma unroll
  for (int q = 0; q < 4; ++q) { S[acc_off(d0, lane, q)] = c0[q]; S[acc_off(d1, lane, q)] = c1[q]; }
}

// pivot wave: factor panel p held in P (rows l + 64 s), diagonal tile in row slot DS; LO:
// slot 0 holds panel rows
template <int DS, bool LO>
__device__ __forceinline__ void factor_panel(double (&P)[2][16], int p, int lane, double* M) {
  const int J0 = 16 * p;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j;
    const double d = rl(P[DS][j], J & 63);
    // v_rsq_f64 (~1e-8 relative) + one Newton step; d <= 0 or NaN gives a NaN L_jj (and NaN
    // below it), which is what the non-PD check after the loop looks for
    const double y = __builtin_amdgcn_rsq(d);
    const double rs = y * fma(-0.5 * d * y, y, 1.5);
    const double ljj = d * rs;
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) {
      const int R = lane + 64 * s;
      const double v = P[s][j] * rs;
      P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
    }
    double* Mj = M + 16 * (j & 1);  // double-buffered: a lagging read never sees column j+1
    {
      const int R = lane + 64 * DS;
      if (R > J && R < J0 + 16) Mj[R - J0] = P[DS][j];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double m1 = 0.0;
    if (j < 15) m1 = rl(P[DS][j], (J + 1) & 63);
#pragma unroll
    for (int c = j + 1; c < 16; ++c) {
#ifdef GPS_V4_PIVOT_LDS
      const double m = c == j + 1 ? m1 : Mj[c];
#else
      const double m = c == j + 1 ? m1 : rl(P[DS][j], (J0 + c) & 63);
#endif
#pragma unroll
      for (int s = LO ? 0 : 1; s < 2; ++s) P[s][c] = fma(-P[s][j], m, P[s][c]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// X_pp = L_pp⁻¹ (16×16 lower; lane c < 16 forms column c by right-looking substitution, so the
// dependent chain is one FMA + one multiply per row) into slot (p,p) and Linv
__device__ __forceinline__ void invert_diag(double* S, double* DG, int p, int lane,
                                            double* Linv, int64_t ldl) {
  const int t = tix(p, p);
  const double lii = S[t * TSZ + (lane & 15) * (TS + 1)];  // lane i: L_ii
  const double rme = 1.0 / lii;
  double acc[16], x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0;
  const int c = lane & 15;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double rk = rl(rme, k);
    x[k] = k < c ? 0.0 : (k == c ? rk : -acc[k] * rk);
#pragma unroll
    for (int i = k + 1; i < 16; ++i) acc[i] = fma(S[t * TSZ + i * TS + k], x[k], acc[i]);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (lane < 16) {
    DG[16 * p + lane] = lii;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      S[t * TSZ + i * TS + lane] = x[i];
      Linv[(int64_t)(16 * p + i) * ldl + 16 * p + lane] = x[i];
    }
  }
}

#ifdef GPS_V4_STAMPS
__device__ long long g_v4_stamps[4][40];  // [wave][event]: tools/diag_bench.cpp timing build only
#define V4_STAMP(ev) do { if (lane == 0) g_v4_stamps[wave][ev] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define V4_STAMP(ev) do { } while (0)
#endif
// tile row of lower tile t (t = i(i+1)/2 + j)
__device__ __forceinline__ constexpr int tile_i(int t) {
  return t < 1 ? 0 : t < 3 ? 1 : t < 6 ? 2 : t < 10 ? 3 : t < 15 ? 4 : t < 21 ? 5 : t < 28 ? 6 : 7;
}

// T_k = Σ_{j=k}^{r-1} L_{r,j} X_{j,k} (two accumulators: the MFMA chain is half as long)
__device__ __forceinline__ d4 inv_row_t(const double* S, int r, int k, int lane) {
  d4 e0 = (d4){0.0, 0.0, 0.0, 0.0}, e1 = e0;
  int j = k;
  for (; j + 1 < r; j += 2) {
    double a0[4], b0[4], a1[4], b1[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      a0[kk] = opnd(S, tix(r, j), lane, kk);
      b0[kk] = S[acc_off(tix(j, k), lane, kk)];
      a1[kk] = opnd(S, tix(r, j + 1), lane, kk);
      b1[kk] = S[acc_off(tix(j + 1, k), lane, kk)];
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) { e0 = mfma(a0[kk], b0[kk], e0); e1 = mfma(a1[kk], b1[kk], e1); }
  }
  if (j < r) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) e0 = mfma(opnd(S, tix(r, j), lane, kk), S[acc_off(tix(j, k), lane, kk)], e0);
  }
  return e0 + e1;
}

// row-7 inverse tasks T_k (k < 7, 7-k tile products each) dealt to 4 waves, 7 products each
__device__ __forceinline__ int tail_k(int wave, int slot) {
  // wave 0: {0}, 1: {1, 6}, 2: {2, 5}, 3: {3, 4}
  return slot == 0 ? wave : (wave == 0 ? -1 : 7 - wave);
}

__global__ __launch_bounds__(256) void potrf_leaf_v4_kernel(
    const double* __restrict__ A, int64_t lda, double* __restrict__ Linv, int64_t ldl,
    double* __restrict__ Lout, int64_t ldlo, double* __restrict__ logdiag, int* info, int base,
    int nreal) {
  __shared__ double S[NT * TSZ];
  __shared__ double M[32];
  __shared__ double DG[128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  V4_STAMP(0);
  // ---- A's lower tiles into LDS (all 18 loads of a thread in flight at once); zeros into
  //      Linv above the tile diagonal
  {
    // thread tid, load m: tile t = 2m + (tid >> 7), pair q = tid & 127 of it (row q >> 3)
    const int hb = tid >> 7, q = tid & 127, r = q >> 3, c2 = (q & 7) * 2;
    dv2 v[18];
#pragma unroll
    for (int m = 0; m < 18; ++m) {
      const int ti = hb ? tile_i(2 * m + 1) : tile_i(2 * m);
      const int tj = hb ? 2 * m + 1 - tix(tile_i(2 * m + 1), 0) : 2 * m - tix(tile_i(2 * m), 0);
      v[m] = *reinterpret_cast<const dv2*>(A + (int64_t)(16 * ti + r) * lda + 16 * tj + c2);
    }
#pragma unroll
    for (int m = 0; m < 18; ++m) {
      const int t = 2 * m + hb;
      S[t * TSZ + r * TS + c2] = v[m].x;
      S[t * TSZ + r * TS + c2 + 1] = v[m].y;
    }
  }
  __syncthreads();
  V4_STAMP(1);

  d4 T[3];                  // the X row in flight: T_k held by the wave that finishes X_{row,k}
  const int uw = wave - 1;  // update-wave index 0..2 in phase A
  for (int p = 0; p < 8; ++p) {
    // ================= phase A: wave 0 factors panel p; waves 1-3: panel p-1 into columns
    //                   >= p+1, X_{p-1,p-1}, T_k of X row p-1
    if (wave == 0) {
      double P[2][16];
      const int t0 = 16 * p;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R = lane + 64 * s;
        const int t = tix(R >> 4, p) * TSZ + (R & 15) * TS;
#pragma unroll
        for (int c = 0; c < 16; ++c) P[s][c] = R >= t0 ? S[t + c] : 0.0;
      }
      if (p < 4) factor_panel<0, true>(P, p, lane, M);
      else factor_panel<1, false>(P, p, lane, M);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R = lane + 64 * s;
        if (R >= t0) {
          const int t = tix(R >> 4, p) * TSZ + (R & 15) * TS;
#pragma unroll
          for (int c = 0; c < 16; ++c) S[t + c] = P[s][c];
        }
        if (Lout) {
          dv2* dst = reinterpret_cast<dv2*>(Lout + (int64_t)R * ldlo + t0);
#pragma unroll
          for (int c = 0; c < 8; ++c)
            dst[c] = R >= t0 ? (dv2){P[s][2 * c], P[s][2 * c + 1]} : (dv2){0.0, 0.0};
        }
      }
    } else if (p >= 1) {
      const int pp = p - 1;
      // wave 1 + pp % 3 inverts L_{pp,pp} (and takes the logs); the bulk tiles go to the
      // other two first, the T_k tasks to all three
      const int winv = pp % 3;
      const int rank = (uw - winv + 3) % 3;  // 0: the inverting wave
      int task = 0;
      for (int j = p + 1; j < 8; ++j)
        for (int i = j; i < 8; ++i, ++task) {
          // deal order: rank 1, rank 2, rank 1, rank 2, ... with every 5th tile to rank 0
          const int who = task % 5 == 4 ? 0 : 1 + ((task - task / 5) & 1);
          if (who == rank) tile_update(S, tix(i, j), tix(i, pp), tix(j, pp), lane);
        }
      if (rank == 0) {
        invert_diag(S, DG, pp, lane, Linv, ldl);
        if (lane < 16) logdiag[16 * pp + lane] = log(DG[16 * pp + lane]);
      }
#pragma unroll
      for (int slot = 0; slot < 3; ++slot) {
        const int k = uw + 3 * slot;
        if (k < pp) T[slot] = inv_row_t(S, pp, k, lane);
      }
    }
    V4_STAMP(2 + 4 * p);
    __syncthreads();
    V4_STAMP(3 + 4 * p);
    // ================= phase B: all 4 waves — panel p into column p+1 (lookahead) and
    //                   X_{p-1,k} = −X_{p-1,p-1} T_k (by the waves holding T_k); X_77 at p = 7
    if (p < 7) {  // tiles (i, p+1), i = p+1..7: wave w takes i = p+1+w and p+5+w
      const int i0 = p + 1 + wave, i1 = p + 5 + wave, tb = tix(p + 1, p);
      if (i1 < 8) tile_update2(S, tix(i0, p + 1), tix(i0, p), tix(i1, p + 1), tix(i1, p), tb, lane);
      else if (i0 < 8) tile_update(S, tix(i0, p + 1), tix(i0, p), tb, lane);
    } else if (wave == 0) {
      invert_diag(S, DG, 7, lane, Linv, ldl);
    }
    if (p >= 1 && wave != 0) {
      const int pp = p - 1, td = tix(pp, pp);
#pragma unroll
      for (int slot = 0; slot < 3; ++slot) {
        const int k = uw + 3 * slot;
        if (k < pp) {
          d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) acc = mfma(-opnd(S, td, lane, kk), T[slot][kk], acc);
          const int tdst = tix(pp, k);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            S[acc_off(tdst, lane, q)] = acc[q];
            Linv[(int64_t)(16 * pp + 4 * q + (lane >> 4)) * ldl + 16 * k + (lane & 15)] = acc[q];
          }
        }
      }
    }
    V4_STAMP(4 + 4 * p);
    __syncthreads();
    V4_STAMP(5 + 4 * p);
  }
  // ================= tail: X row 7 (T_k on all 4 waves, 7 tile products each), then finish
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int k = tail_k(wave, slot);
    if (k >= 0) T[slot] = inv_row_t(S, 7, k, lane);
  }
  V4_STAMP(37);
  __syncthreads();  // (X row 6 and X_77 were final before; only the reads above precede this)
  V4_STAMP(38);
  {
    const int td = tix(7, 7);
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int k = tail_k(wave, slot);
      if (k >= 0) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) acc = mfma(-opnd(S, td, lane, kk), T[slot][kk], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          Linv[(int64_t)(16 * 7 + 4 * q + (lane >> 4)) * ldl + 16 * k + (lane & 15)] = acc[q];
      }
    }
  }
  V4_STAMP(39);
  if (tid < 128) {
    // first non-positive pivot (torch.potrf's leading-minor index): a bad pivot makes its
    // L_ii NaN and poisons every later one, so the minimum flagged index is the first
    const double dg = DG[tid];
    if (!(dg > 0.0) && tid < nreal) atomicMin(info, base + tid + 1);
  } else if (tid >= 240) {
    logdiag[112 + tid - 240] = log(DG[112 + tid - 240]);
  }
  {  // zeros above the tile diagonal of Linv: the 28 upper tiles, 14 dv2 per thread
    const int hb = tid >> 7, q = tid & 127, r = q >> 3, c2 = (q & 7) * 2;
#pragma unroll
    for (int m = 0; m < 14; ++m) {
      const int u = 2 * m + hb;  // upper tile u: (i, j), i < j, row-major over i
      const int ui = u < 7 ? 0 : u < 13 ? 1 : u < 18 ? 2 : u < 22 ? 3 : u < 25 ? 4 : u < 27 ? 5 : 6;
      const int ustart = ui * 7 - ui * (ui - 1) / 2;  // first upper tile of row ui
      const int uj = ui + 1 + (u - ustart);
      *reinterpret_cast<dv2*>(Linv + (int64_t)(16 * ui + r) * ldl + 16 * uj + c2) = (dv2){0.0, 0.0};
    }
  }
  V4_STAMP(36);
}
}  // namespace v4

int g_leaf_v4 = 1;  // GPS_OPT_LEAF: 1 the v4 MFMA leaf, 0 the v3 register-blocked leaf

hipError_t launch_potrf_leaf(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                             int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                             hipStream_t s) {
  if ((lda & 1) || (ldl & 1) || (Lout && (ldlo & 1))) return hipErrorInvalidValue;
  if (g_leaf_v4) {
    hipLaunchKernelGGL(v4::potrf_leaf_v4_kernel, dim3(1), dim3(256), 0, s, A, lda, Linv, ldl, Lout,
                       ldlo, logdiag, info, base, nreal);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(potrf_diag_v3_kernel, dim3(1), dim3(64 * V3_WAVES), 0, s, A, lda, Linv, ldl,
                     Lout, ldlo, logdiag, info, base, nreal);
  return hipGetLastError();
}

}  // namespace gps
