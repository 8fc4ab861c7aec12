// Diagonal-block kernel of the blocked Cholesky (replaces LAPACK ?potrf behind
// torch.potrf, KF:26 / KF:332) fused with the block's triangular inverse: the leaf of the
// recursive factorisation (csrc/api.hip potrf_inv_rec), one 128×128 block per launch.
// (The round-1 register-blocked VALU kernel, 51 µs, is kept outside the library as the A/B
// baseline: tools/leaf_v3.hip, tools/diag_bench.cpp.)
#include "gps_internal.h"

namespace gps {

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
__device__ __forceinline__ void factor_panel(double (&P)[2][16], int p, int lane) {
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
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double m1 = 0.0;
    if (j < 15) m1 = rl(P[DS][j], (J + 1) & 63);
#pragma unroll
    for (int c = j + 1; c < 16; ++c) {
      const double m = c == j + 1 ? m1 : rl(P[DS][j], (J0 + c) & 63);
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
  __shared__ double DG[128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
      if (p < 4) factor_panel<0, true>(P, p, lane);
      else factor_panel<1, false>(P, p, lane);
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
    __syncthreads();
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
    __syncthreads();
  }
  // ================= tail: X row 7 (T_k on all 4 waves, 7 tile products each), then finish
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int k = tail_k(wave, slot);
    if (k >= 0) T[slot] = inv_row_t(S, 7, k, lane);
  }
  __syncthreads();  // (X row 6 and X_77 were final before; only the reads above precede this)
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
}
}  // namespace v4

hipError_t launch_potrf_leaf(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                             int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                             hipStream_t s) {
  if ((lda & 1) || (ldl & 1) || (Lout && (ldlo & 1))) return hipErrorInvalidValue;
  hipLaunchKernelGGL(v4::potrf_leaf_v4_kernel, dim3(1), dim3(256), 0, s, A, lda, Linv, ldl, Lout,
                     ldlo, logdiag, info, base, nreal);
  return hipGetLastError();
}

}  // namespace gps
