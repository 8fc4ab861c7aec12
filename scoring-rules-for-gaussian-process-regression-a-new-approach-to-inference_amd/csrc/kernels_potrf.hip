// Diagonal-block kernel of the blocked Cholesky (replaces LAPACK ?potrf behind
// torch.potrf, KF:26 / KF:332) fused with the block's triangular inverse: the leaf of the
// recursive factorisation (csrc/api.hip potrf_inv_rec), one 128×128 block per launch.
// (The round-1 register-blocked VALU kernel, 51 µs, is kept outside the library as the A/B
// baseline: tools/leaf_v3.hip, tools/diag_bench.cpp.)
#include <algorithm>
#include <queue>
#include <vector>

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
// Coherent (write-through, L1-bypassing: `sc1`) element access for data handed between the
// workgroups of one launch (the persistent factorisation below); plain access otherwise.
template <bool COH>
__device__ __forceinline__ void st_d(double* p, double v) {
  if constexpr (COH)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                       (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
template <bool COH>
__device__ __forceinline__ void st_d2(double* p, dv2 v) {
  if constexpr (COH) {
    st_d<true>(p, v.x);
    st_d<true>(p + 1, v.y);
  } else {
    *reinterpret_cast<dv2*>(p) = v;
  }
}
template <bool COH>
__device__ __forceinline__ dv2 ld_d2(const double* p) {
  if constexpr (COH) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (dv2){__longlong_as_double((long long)a), __longlong_as_double((long long)b)};
  } else {
    return *reinterpret_cast<const dv2*>(p);
  }
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

// lane c of every 16-lane row gets x from lane C of its own row (v_mov_b64 row_newbcast:C)
template <int C>
__device__ __forceinline__ double row_bcast(double x) {
  long long v = __double_as_longlong(x), old = 0;
  return __longlong_as_double(__builtin_amdgcn_update_dpp(old, v, 0x150 + C, 0xf, 0xf, true));
}

// pivot wave: factor panel p held in P (rows l + 64 s), diagonal tile in row slot DS; LO:
// slot 0 holds panel rows.  Per column j: the pivot by v_readlane, v_rsq_f64 + one Newton step;
// the next column's multiplier (the dependent chain) by v_readlane; the rest of column j's
// multipliers L[J0+c][j] from ONE copy of the diagonal tile's column in every 16-lane row
// (two ds_bpermute) and a 64-bit DPP row broadcast each — the v_readlane pair per multiplier
// this replaces was the panel's issue bound (tools/panel_probe.hip v7 vs v8: 3.8k vs 4.3k cycles
// with one row slot).  Every element gets the same FMAs in the same order: bitwise the same L.
template <int DS, bool LO>
__device__ __forceinline__ void factor_panel(double (&P)[2][16], int p, int lane) {
  const int J0 = 16 * p;
  const int src = 4 * ((J0 & 63) + (lane & 15));  // bpermute byte address: the diagonal row
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j;
    const double d = rl(P[DS][j], J & 63);
    // v_rsq_f64 (~1e-8 relative) + one Newton step leaves 1/√d ~3 ulp off (1.5e0² + the step's
    // roundings); a second, residual-corrected step (h = 1 − d·r² by FMA, r += r·h/2) brings it to
    // ~1 ulp, as LAPACK's sqrt and reciprocal.  Round 6: the one-step pivots made the FITC B
    // factor's inverse 3-10x less accurate than LAPACK's at cond(B) 7e7.  d <= 0 or
    // NaN gives a NaN L_jj (and NaN below it), which is what the non-PD check after the loop
    // looks for
    const double y = __builtin_amdgcn_rsq(d);
    const double r1 = y * fma(-0.5 * d * y, y, 1.5);
    const double rs = fma(0.5 * r1, fma(-d * r1, r1, 1.0), r1);
    const double ljj = d * rs;
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) {
      const int R = lane + 64 * s;
      const double v = P[s][j] * rs;
      P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
    }
    if (j == 15) break;
    const double pj = P[DS][j];
    const int clo = __builtin_amdgcn_ds_bpermute(src, __double2loint(pj));
    const int chi = __builtin_amdgcn_ds_bpermute(src, __double2hiint(pj));
    const double m1 = rl(pj, (J + 1) & 63);
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) P[s][j + 1] = fma(-P[s][j], m1, P[s][j + 1]);
    const double col = __hiloint2double(chi, clo);
#define GPS_PANEL_UPD(C)                                                                  \
    if (C > j + 1) {                                                                      \
      const double m = row_bcast<C>(col);                                                 \
      _Pragma("unroll") for (int s = LO ? 0 : 1; s < 2; ++s) P[s][C] = fma(-P[s][j], m, P[s][C]); \
    }
    GPS_PANEL_UPD(2) GPS_PANEL_UPD(3) GPS_PANEL_UPD(4) GPS_PANEL_UPD(5) GPS_PANEL_UPD(6)
    GPS_PANEL_UPD(7) GPS_PANEL_UPD(8) GPS_PANEL_UPD(9) GPS_PANEL_UPD(10) GPS_PANEL_UPD(11)
    GPS_PANEL_UPD(12) GPS_PANEL_UPD(13) GPS_PANEL_UPD(14) GPS_PANEL_UPD(15)
#undef GPS_PANEL_UPD
  }
}

// X_pp = L_pp⁻¹ (16×16 lower; lane c < 16 forms column c by right-looking substitution, so the
// dependent chain is one FMA + one multiply per row) into slot (p,p) and Linv
template <bool COH>
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
      st_d<COH>(Linv + (int64_t)(16 * p + i) * ldl + 16 * p + lane, x[i]);
    }
  }
}

// tile row of lower tile t (t = i(i+1)/2 + j)
__device__ __forceinline__ constexpr int tile_i(int t) {
  return t < 1 ? 0 : t < 3 ? 1 : t < 6 ? 2 : t < 10 ? 3 : t < 15 ? 4 : t < 21 ? 5 : t < 28 ? 6 : 7;
}

// Phase A's trailing tiles per (step p, rank of the update wave): every 5th tile to the wave that
// also inverts L_{p-1,p-1}, the rest alternating over the other two; a table (dwords: dst | a << 8
// | b << 16, scalar loads) so that a wave can batch its tiles.  A tile update cost ~1k cycles
// one at a time (its LDS reads, then a 4-MFMA chain of 64 cycles each — one wave per SIMD issues
// f64 MFMAs at the full rate, dependent or not: tools/mfma_f64_rate.hip — then the result wait
// before the writes); three tiles per group overlap those latencies (phase A of the first steps
// 10.3k -> 7.6k cycles, tools/leaf_probe.hip).
struct Deal {
  int n[8][3];
  unsigned int t[8][3][12];
};
constexpr Deal make_deal() {
  Deal d{};
  for (int p = 1; p < 8; ++p) {
    int task = 0;
    for (int j = p + 1; j < 8; ++j)
      for (int i = j; i < 8; ++i, ++task) {
        const int who = task % 5 == 4 ? 0 : 1 + ((task - task / 5) & 1);
        d.t[p][who][d.n[p][who]++] =
            (unsigned)tix(i, j) | (unsigned)tix(i, p - 1) << 8 | (unsigned)tix(j, p - 1) << 16;
      }
  }
  return d;
}
__constant__ Deal g_deal = make_deal();

// S_dst[u] −= L_a[u] L_b[u]ᵀ for up to G tiles of the list: every LDS read of the group, then the
// MFMAs (G independent chains, each tile's in tile_update's order: the same bits), then the writes
template <int G>
__device__ __forceinline__ void tile_update_group(double* S, const unsigned int* tl, int cnt, int lane) {
  d4 c[G];
  double a[G][4], b[G][4];
  int td[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    if (u < cnt) {
      const unsigned w = tl[u];
      td[u] = w & 255;
      const int ta = (w >> 8) & 255, tb = w >> 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) c[u][q] = S[acc_off(td[u], lane, q)];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) { a[u][kk] = -opnd(S, ta, lane, kk); b[u][kk] = opnd(S, tb, lane, kk); }
    }
  }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int u = 0; u < G; ++u)
      if (u < cnt) c[u] = mfma(a[u][kk], b[u][kk], c[u]);
#pragma unroll
  for (int u = 0; u < G; ++u)
    if (u < cnt)
#pragma unroll
      for (int q = 0; q < 4; ++q) S[acc_off(td[u], lane, q)] = c[u][q];
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

// The leaf as a device function of one 256-thread workgroup: the stand-alone kernel below
// (COH = false) and the persistent factorisation's LEAF task (COH = true: A read and L⁻¹ written
// coherently, since other workgroups of the same launch produce / consume them).  S, DG: LDS.
template <bool COH>
__device__ __forceinline__ void leaf_body(const double* __restrict__ A, int64_t lda,
                                          double* __restrict__ Linv, int64_t ldl,
                                          double* __restrict__ Lout, int64_t ldlo,
                                          double* __restrict__ logdiag, int* info, int base,
                                          int nreal, double* S, double* DG) {
  const int tid = threadIdx.x, lane = tid & 63;
  // the wave index as a scalar: its branches and the tile-table loads then stay on the scalar unit
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
      v[m] = ld_d2<COH>(A + (int64_t)(16 * ti + r) * lda + 16 * tj + c2);
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
        if (Lout && R >= t0) {
          dv2* dst = reinterpret_cast<dv2*>(Lout + (int64_t)R * ldlo + t0);
#pragma unroll
          for (int c = 0; c < 8; ++c) dst[c] = (dv2){P[s][2 * c], P[s][2 * c + 1]};
        }
      }
    } else if (p >= 1) {
      const int pp = p - 1;
      // wave 1 + pp % 3 inverts L_{pp,pp} (and takes the logs); the bulk tiles go to the
      // other two first, the T_k tasks to all three
      const int winv = pp % 3;
      const int rank = (uw - winv + 3) % 3;  // 0: the inverting wave
      const int nt = g_deal.n[p][rank];
      for (int g0 = 0; g0 < nt; g0 += 3) tile_update_group<3>(S, g_deal.t[p][rank] + g0, nt - g0, lane);
      if (rank == 0) {
        invert_diag<COH>(S, DG, pp, lane, Linv, ldl);
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
      invert_diag<COH>(S, DG, 7, lane, Linv, ldl);
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
            st_d<COH>(Linv + (int64_t)(16 * pp + 4 * q + (lane >> 4)) * ldl + 16 * k + (lane & 15),
                      acc[q]);
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
          st_d<COH>(Linv + (int64_t)(16 * 7 + 4 * q + (lane >> 4)) * ldl + 16 * k + (lane & 15),
                    acc[q]);
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
  // (the 28 16×16 tiles above the tile diagonal of Linv, and Lout's rows above each column
  // panel, are not written: every caller zeroes the factor buffers when it (re)allocates them and
  // nothing writes there afterwards — round 4: 57 KB less write-through traffic to drain at the
  // end of every persistent LEAF)
}

__global__ __launch_bounds__(256) void potrf_leaf_v4_kernel(
    const double* __restrict__ A, int64_t lda, double* __restrict__ Linv, int64_t ldl,
    double* __restrict__ Lout, int64_t ldlo, double* __restrict__ logdiag, int* info, int base,
    int nreal) {
  __shared__ double S[NT * TSZ];
  __shared__ double DG[128];
  leaf_body<false>(A, lda, Linv, ldl, Lout, ldlo, logdiag, info, base, nreal, S, DG);
}
}  // namespace v4

// ---------------------------------------------------------------------------
// Persistent tiled factorisation of a diagonal block of T ≤ 64 tiles (128 columns each): L and
// L⁻¹ in ONE launch.  The bottom of the recursion (potrf_inv_rec in api.hip) used to be a chain
// of ~7 dependent launches per 128 columns (leaf, the TRSM / SYRK / T / TRMM products of every
// recursion level), each a few µs of work behind a ~5 µs launch boundary with most of the chip
// idle; here one workgroup per CU pulls tasks from a device queue, waits for their inputs through
// per-tile arrival counters and publishes its outputs write-through, so the chain costs the
// leaves plus a cross-workgroup hand-off (~µs) per dependent product.
//
// Tasks (tile indices in the block; L_ik lands in A_ik, X = L⁻¹ in Linv):
//   LEAF(k)        [L_kk, X_kk] = leaf(A_kk)                                  (one workgroup)
//   TRSM(i,k)      L_ik  = A_ik · X_kkᵀ                        i > k          (4 row strips)
//   UPD(i,j,k)     A_ij −= L_ik · L_jkᵀ                        i ≥ j > k      (4 row strips)
//   UPDX(i,k,j)    S_ik (+)= L_ij · X_jk  (first term: =)      i > j ≥ k      (4 row strips)
//   FIN(i,k)       X_ik  = −X_ii · S_ik   (in place)           i > k          (4 column strips)
// (right-looking Cholesky; the inverse right-looking too: X_ik = −X_ii Σ_{j=k}^{i−1} L_ij X_jk,
// S_ik accumulated in X's own tile).  Each strip task runs on 4 waves, each a 32×32 block of
// v_mfma_f64_16x16x4 with its operands streamed from L2 (no LDS), the K range clipped to the
// triangular operand's nonzeros.  Arrival counters per tile: A-side acnt[i][j] (+4 per UPD, +4
// per TRSM, +1 per LEAF) and X-side xcnt[i][k] (+4 per UPDX / FIN, +1 per LEAF); a task polls
// the counts it needs (one lane, relaxed agent-scope loads, bounded) — every input of a task
// was written by tasks earlier in the queue, so the queue order (a topological order, host
// side: dag_task_list) guarantees progress for any residency.  Hand-offs follow the
// write-through form of cdna_hip_programming.md §6 Guideline 16: payload stores `sc1`, every
// wave drains (vmcnt 0), barrier, one relaxed agent atomic add; consumers load `sc1`.
namespace dag {
using v4::d4;
using v4::dv2;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
constexpr int NP = 4;        // strips per tile task
constexpr int NPF_TRSM = 8;  // parts of a fine TRSM (16-row strips)
constexpr int NPF_UPD = 16;  // parts of a fine UPD (16 × 64 blocks)
constexpr int U = 16;        // arrivals per finished tile task: 4 per strip, 2 / 1 per fine part
constexpr int AUX_SC1 = 16;  // cache-policy bits of the buffer intrinsics: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ dv2 ld128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX_SC1));
}
__device__ __forceinline__ double ld64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX_SC1));
}
__device__ __forceinline__ void st64(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, off, 0, AUX_SC1);
}
__device__ __forceinline__ int ld_cnt(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wave: acc = A (32 rows, k in [kb, ke), lda) · B, B stored [k][j] (BT = false, 32 columns)
// or [j][k] (BT = true, 32 rows); operand fragments straight from L2 (sc1) in groups of G
// 16-deep chunks, one group ahead of the MFMAs (the layout of gemm_f64_small_kernel).  A chunk is
// 32 VGPRs per lane, so G bounds how many loads are in flight per wave: the operands were just
// handed over (written through by another workgroup, often on another XCD), so every group pays a
// full fabric latency, and with K = 128 at G = 2 the strip waited four of them (9-12 µs per strip
// task against 3.4 µs of MFMA, profiles/r3_dag_trace20.txt).
template <bool BT, int G>
__device__ __forceinline__ void wave_gemm32(const double* Ap, int64_t lda, const double* Bp,
                                            int64_t ldb, int kb, int ke, d4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t ra = rsrc(Ap, (uint32_t)(32 * lda * 8));
  const __amdgpu_buffer_rsrc_t rb = rsrc(Bp, (uint32_t)((BT ? 32 : 128) * ldb * 8));
  typedef double Frag[G][2][4];  // [chunk in group][16-block][k step]
  const int nc = (ke - kb) / 16;
  auto load_group = [&](int c, Frag& a, Frag& b) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (c + u >= nc) break;  // wave-uniform
      const int k = kb + 16 * (c + u) + 4 * g;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t oa = (uint32_t)(((int64_t)(16 * i + r) * lda + k) * 8);
        const dv2 a0 = ld128(ra, oa), a1 = ld128(ra, oa + 16);
        a[u][i][0] = a0.x; a[u][i][1] = a0.y; a[u][i][2] = a1.x; a[u][i][3] = a1.y;
        if constexpr (BT) {
          const uint32_t ob = (uint32_t)(((int64_t)(16 * i + r) * ldb + k) * 8);
          const dv2 b0 = ld128(rb, ob), b1 = ld128(rb, ob + 16);
          b[u][i][0] = b0.x; b[u][i][1] = b0.y; b[u][i][2] = b1.x; b[u][i][3] = b1.y;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            b[u][i][e] = ld64(rb, (uint32_t)(((int64_t)(k + e) * ldb + 16 * i + r) * 8));
        }
      }
    }
  };
  auto mma_group = [&](int c, const Frag& a, const Frag& b) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (c + u >= nc) break;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][i][kk], b[u][j][kk], acc[i][j], 0, 0, 0);
    }
  };
  {
    Frag fa0, fb0, fa1, fb1;
    int c = 0;
    if (c < nc) load_group(c, fa0, fb0);
    while (c < nc) {
      if (c + G < nc) load_group(c + G, fa1, fb1);
      mma_group(c, fa0, fb0);
      c += G;
      if (c >= nc) break;
      if (c + G < nc) load_group(c + G, fa0, fb0);
      mma_group(c, fa1, fb1);
      c += G;
    }
  }
}

struct Strip {          // one wave's 32×32 block of a strip task
  const double* A; int64_t lda;
  const double* B; int64_t ldb; int bt;
  double* C; int64_t ldc;
  double* C2; int64_t ldc2;   // optional plain copy of the result (L into Lout)
  double alpha, beta;
  int kb, ke, active;
};

// all four waves: compute, barrier (in-place tasks: every read of the strip precedes every
// write), then write-through stores
template <int G>
__device__ __forceinline__ void run_strip(const Strip& s) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t rc = rsrc(s.C, (uint32_t)(32 * s.ldc * 8));
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  double cold[2][2][4];
  if (s.active) {
    if (s.beta != 0.0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            cold[i][j][e] = ld64(rc, (uint32_t)(((int64_t)(16 * i + g + 4 * e) * s.ldc + 16 * j + r) * 8));
    }
    if (s.bt) wave_gemm32<true, G>(s.A, s.lda, s.B, s.ldb, s.kb, s.ke, acc);
    else wave_gemm32<false, G>(s.A, s.lda, s.B, s.ldb, s.kb, s.ke, acc);
  }
  __syncthreads();
  if (!s.active) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        double v = s.alpha * acc[i][j][e];
        if (s.beta != 0.0) v = fma(s.beta, cold[i][j][e], v);
        const int64_t row = 16 * i + g + 4 * e, col = 16 * j + r;
        st64(rc, (uint32_t)((row * s.ldc + col) * 8), v);
        if (s.C2) s.C2[row * s.ldc2 + col] = v;
      }
}

// Fine parts of the two tile tasks on the leaf chain, TRSM(k+1,k) and UPD(k+1,k+1,k) (round 4):
// LEAF(k) -> TRSM(k+1,k) -> UPD(k+1,k+1,k) -> LEAF(k+1) ran 9.5 + 11.7 µs of strip tasks per
// 128 columns (profiles/r3_dag_trace20_rank.txt), each wave a 32×32 block with K = 128: 128
// dependent-group MFMAs (3.4 µs) behind several fabric round trips.  A fine part gives each wave
// 16×16 blocks (TRSM: 16 rows, the column blocks w and 7 − w, whose triangular K ranges sum to
// the same 144; UPD: one block), every operand chunk in flight before the first MFMA.  The
// in-place TRSM keeps whole rows per workgroup (its A strip is read across all columns).  The
// MFMA sequence per output element is the strip task's (chunks ascending, the same k
// permutation): the same bits, bar the all-zero chunks above X_kk's diagonal the strip adds.
// one wave: acc[c] = A (16 rows, k < ke[c]) · B_cᵀ (B_c: 16 rows, [j][k]), c < 2, ke ≤ 128
__device__ __forceinline__ void wave_gemm16(const double* Ap, int64_t lda, const double* B0,
                                            const double* B1, int64_t ldb, int ke0, int ke1,
                                            d4 (&acc)[2]) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t ra = rsrc(Ap, (uint32_t)(16 * lda * 8));
  const __amdgpu_buffer_rsrc_t rb0 = rsrc(B0, (uint32_t)(16 * ldb * 8));
  const __amdgpu_buffer_rsrc_t rb1 = rsrc(B1 ? B1 : B0, (uint32_t)(16 * ldb * 8));
  const int kmax = ke0 > ke1 ? ke0 : ke1;
  double a[8][4], b0[8][4], b1[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int k = 16 * u + 4 * g;
    const uint32_t o = (uint32_t)(((int64_t)r * lda + k) * 8), ob = (uint32_t)(((int64_t)r * ldb + k) * 8);
    if (16 * u < kmax) {
      const dv2 x0 = ld128(ra, o), x1 = ld128(ra, o + 16);
      a[u][0] = x0.x; a[u][1] = x0.y; a[u][2] = x1.x; a[u][3] = x1.y;
    }
    if (16 * u < ke0) {
      const dv2 x0 = ld128(rb0, ob), x1 = ld128(rb0, ob + 16);
      b0[u][0] = x0.x; b0[u][1] = x0.y; b0[u][2] = x1.x; b0[u][3] = x1.y;
    }
    if (16 * u < ke1) {
      const dv2 x0 = ld128(rb1, ob), x1 = ld128(rb1, ob + 16);
      b1[u][0] = x0.x; b1[u][1] = x0.y; b1[u][2] = x1.x; b1[u][3] = x1.y;
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (16 * u < ke0) acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][kk], b0[u][kk], acc[0], 0, 0, 0);
      if (16 * u < ke1) acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][kk], b1[u][kk], acc[1], 0, 0, 0);
    }
}

// one fine part on all four waves: each wave's (up to) two 16×16 output blocks of C rows
// [0, 16), columns c0·16.. and c1·16.. (c < 0: none); barrier before the write-through stores
// (the TRSM reads its strip in place)
struct Fine {
  const double* A; int64_t lda;      // the strip's 16 rows, k from 0
  const double* B; int64_t ldb;      // B block c at B + 16c·ldb (rows [j][k])
  double* C; int64_t ldc;            // C block c at C + 16c
  double* C2; int64_t ldc2;          // optional plain copy (L into Lout)
  double alpha, beta;
  int c0, c1, ke0, ke1;              // per wave
};
__device__ __forceinline__ void run_fine(const Fine& s) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  d4 acc[2] = {(d4){0.0, 0.0, 0.0, 0.0}, (d4){0.0, 0.0, 0.0, 0.0}};
  const int cs[2] = {s.c0, s.c1};
  double cold[2][4];
  const __amdgpu_buffer_rsrc_t rc = rsrc(s.C, (uint32_t)(16 * s.ldc * 8));
  if (s.beta != 0.0) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (cs[c] >= 0)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          cold[c][e] = ld64(rc, (uint32_t)(((int64_t)(g + 4 * e) * s.ldc + 16 * cs[c] + r) * 8));
  }
  const int ke0 = s.c0 >= 0 ? s.ke0 : 0, ke1 = s.c1 >= 0 ? s.ke1 : 0;
  if (ke0 | ke1)
    wave_gemm16(s.A, s.lda, s.B + (int64_t)16 * (s.c0 >= 0 ? s.c0 : 0) * s.ldb,
                s.c1 >= 0 ? s.B + (int64_t)16 * s.c1 * s.ldb : nullptr, s.ldb, ke0, ke1, acc);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (cs[c] < 0) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      double v = s.alpha * acc[c][e];
      if (s.beta != 0.0) v = fma(s.beta, cold[c][e], v);
      const int64_t row = g + 4 * e, col = 16 * cs[c] + r;
      st64(rc, (uint32_t)((row * s.ldc + col) * 8), v);
      if (s.C2) s.C2[row * s.ldc2 + col] = v;
    }
  }
}

// Counters: cnt[0] the queue head, cnt[1] the workgroups out, cnt[16..] the arrival counters —
// zero at launch, zero again when the last workgroup leaves.
// TRACE: per queue slot t, trace[4t..4t+3] = {fetched, inputs ready, outputs drained} in 100 MHz
// s_memrealtime ticks and (blockIdx << 8 | XCC id) — the diagnostics launch (tools/dag_bench.cpp)
// (GPS_DAG_WAVES_PER_EU: a build knob for tools/dag_bench.cpp A/B runs — 2 asks the compiler for
// two workgroups per CU, i.e. ≤ 256 registers per lane, at the cost of scratch spills)
#ifndef GPS_DAG_WAVES_PER_EU
#define GPS_DAG_WAVES_PER_EU 1
#endif
template <bool TRACE, int G>
__global__ __launch_bounds__(256, GPS_DAG_WAVES_PER_EU) void potrf_dag_kernel(DagParams p) {
  __shared__ double S[v4::NT * v4::TSZ];
  __shared__ double DG[128];
  __shared__ unsigned int sh[3];  // [task word, abort, queue slot]
  const int tid = threadIdx.x;
  const int T = p.T;
  int* head = p.cnt;
  int* acnt = p.cnt + 16;
  int* xcnt = acnt + T * T;
  int* err = p.info + 1;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Every branch that leaves the loop or spins is wave-uniform (readfirstlane): a loop exit the
  // compiler must treat as divergent lets it rotate the `tid == 0` parts into another loop level
  // than the rest of the wave, which then runs tasks without the lane that fetched them.
  // The previous task's arrivals are published in the same lane-0 region that fetches the next
  // task (one divergent region per iteration, right after the barrier that ends the task): two
  // adjacent `tid == 0` regions around the loop latch get jump-threaded into a second back edge
  // that only lane 0 takes, and the SIMT lowering then loops the other lanes over a stale task.
  int* out = nullptr;
  int* out2 = nullptr;
  int inc = 0;                         // the arrival the current task adds to *out
  unsigned long long* trow = nullptr;  // TRACE: the current slot's record
  int ndone = 0;                       // queue slots this workgroup completed
  // row signal of the current task for a dependent row-norm launch (p.sig): row | need << 8 —
  // need = the FIN strips of the row (NP per FIN(i, k), k < i), 0 for LEAF(0); −1: none
  int srow = -1;
  if (p.sig && tid == 0)
    __hip_atomic_fetch_add(p.sig + kSigStarted, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (tid == 0) {
      if constexpr (TRACE) {  // (the previous task's "done" stamp lives here for the same reason)
        if (trow) trow[2] = __builtin_amdgcn_s_memrealtime();
      }
      if (out) __hip_atomic_fetch_add(out, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (out2) __hip_atomic_fetch_add(out2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (srow >= 0) {  // (the strip's stores drained before the barrier, as for the arrivals)
        const int row = srow & 255, need = srow >> 8;
        if (need == 0 || __hip_atomic_fetch_add(p.sig + kSigRowCnt + row, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) == need - 1)
          __hip_atomic_store(p.sig + kSigRdy + row, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int t = __hip_atomic_fetch_add(head, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sh[0] = t < p.ntasks ? p.tasks[t] : 0xffffffffu;
      sh[1] = 0;
      sh[2] = (unsigned int)t;
    }
    __syncthreads();
    const unsigned int w = __builtin_amdgcn_readfirstlane(sh[0]);
    if (w == 0xffffffffu) break;
    if constexpr (TRACE) {
      trow = p.trace + 4 * (int64_t)__builtin_amdgcn_readfirstlane(sh[2]);
      if (tid == 0) {
        unsigned int xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        trow[0] = __builtin_amdgcn_s_memrealtime();
        trow[3] = (unsigned long long)blockIdx.x << 8 | (xcc & 15);
      }
    }
    const int type = w & 7, part = (w >> 3) & 15, fine = (w >> 7) & 1, ti = (w >> 8) & 255,
              tj = (w >> 16) & 255, tk = (w >> 24) & 255;
    // ---- the counts this task needs (see the header); up to three, polled by wave 0 (every
    //      lane loads the same word; the exit test is taken on lane 0's view)
    if (wave == 0) {
      const int* c0 = nullptr; const int* c1 = nullptr; const int* c2 = nullptr;
      int v0 = 0, v1 = 0, v2 = 0;
      switch (type) {
        case 0:  // LEAF(k = ti)
          c0 = acnt + ti * T + ti; v0 = U * ti;
          break;
        case 1:  // TRSM(i, k): A_ik final, X_kk from LEAF(k)
          c0 = acnt + ti * T + tk; v0 = U * tk;
          c1 = xcnt + tk * T + tk; v1 = 1;
          break;
        case 2:  // UPD(i, j, k)
          c0 = acnt + ti * T + tk; v0 = U * (tk + 1);
          c1 = acnt + tj * T + tk; v1 = U * (tk + 1);
          c2 = acnt + ti * T + tj; v2 = U * tk;
          break;
        case 3:  // UPDX(i, k, j): L_ij final, X_jk final, S_ik's earlier terms
          c0 = acnt + ti * T + tj; v0 = U * (tj + 1);
          c1 = xcnt + tj * T + tk; v1 = tj == tk ? 1 : U * (tj - tk + 1);
          c2 = xcnt + ti * T + tk; v2 = U * (tj - tk);
          break;
        case 4:  // FIN(i, k)
          c0 = xcnt + ti * T + tk; v0 = U * (ti - tk);
          c1 = xcnt + ti * T + ti; v1 = 1;
          break;
        default: break;
      }
      if (!c1) { c1 = c0; v1 = v0; }
      if (!c2) { c2 = c0; v2 = v0; }
      // A lost dependency is declared only after spin_ticks of wall clock with no movement of
      // the polled counts AND at least kMinPolls polls: time this queue spends descheduled (the
      // GPU time-sliced to another process) advances the clock but not the poll count.
      constexpr unsigned int kMinPolls = 100000;
      unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned int ab = 0, polls = 0;
      int seen = -1;
      for (;;) {
        const int a0 = ld_cnt(c0), a1 = ld_cnt(c1), a2 = ld_cnt(c2), e = ld_cnt(err);
        if (__builtin_amdgcn_readfirstlane((a0 >= v0 && a1 >= v1 && a2 >= v2) ? 1 : 0)) break;
        if (__builtin_amdgcn_readfirstlane(e != 0x7f7f7f7f ? 1 : 0)) { ab = 1; break; }
        const int s = __builtin_amdgcn_readfirstlane(a0 + a1 + a2);
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (s != seen) {  // progress: restart the clock
          seen = s;
          t0 = now;
          polls = 0;
        } else if (++polls > kMinPolls && now - t0 > p.spin_ticks) {
          if (tid == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ab = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (tid == 0) sh[1] = ab;
      // agent-scope acquire: the producers' payload (stored write-through, drained, then the
      // relaxed agent-scope arrival) is visible to every load after this fence by the memory
      // model itself — the other waves are ordered behind it by the workgroup barrier below —
      // not only by the sc1 loads happening to miss the CU cache.
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(sh[1])) break;
    if constexpr (TRACE) {
      if (tid == 0) trow[1] = __builtin_amdgcn_s_memrealtime();
    }
    const int64_t lda = p.lda, ldl = p.ldl;
    out2 = nullptr;
    srow = !p.sig ? -1 : type == 4 ? ti | (NP * ti) << 8 : (type == 0 && ti == 0) ? 0 : -1;
    if (type == 0) {
      const int64_t o = (int64_t)128 * ti;
      v4::leaf_body<true>(p.A + o * lda + o, lda, p.Linv + o * ldl + o, ldl,
                          p.Lout ? p.Lout + o * p.ldlo + o : nullptr, p.ldlo, p.logdiag + o,
                          p.info, p.base + (int)o, p.nreal - (int)o, S, DG);
      out = acnt + ti * T + ti;
      out2 = xcnt + ti * T + ti;
      inc = 1;
    } else if (fine) {
      Fine f;
      const int64_t R = 128 * (int64_t)ti, K = 128 * (int64_t)tk;
      f.C2 = nullptr;
      f.ldc2 = 0;
      if (type == 1) {  // TRSM(k+1, k): rows 16·part.. of L_ik = A_ik · X_kkᵀ, column blocks w, 7 − w
        const int64_t r0 = R + 16 * part;
        f.A = p.A + r0 * lda + K; f.lda = lda;
        f.B = p.Linv + K * ldl + K; f.ldb = ldl;
        f.C = p.A + r0 * lda + K; f.ldc = lda;
        if (p.Lout) { f.C2 = p.Lout + r0 * p.ldlo + K; f.ldc2 = p.ldlo; }
        f.alpha = 1.0; f.beta = 0.0;
        f.c0 = wave; f.c1 = 7 - wave; f.ke0 = 16 * (wave + 1); f.ke1 = 16 * (8 - wave);
        inc = U / NPF_TRSM;
        out = acnt + ti * T + tk;
      } else {  // UPD(k+1, k+1, k): row block part >> 1, column block 4·(part & 1) + w (lower only)
        const int64_t J = 128 * (int64_t)tj, rb = part >> 1, cb = 4 * (part & 1) + wave;
        f.A = p.A + (R + 16 * rb) * lda + K; f.lda = lda;
        f.B = p.A + J * lda + K; f.ldb = lda;
        f.C = p.A + (R + 16 * rb) * lda + J; f.ldc = lda;
        f.alpha = -1.0; f.beta = 1.0;
        f.c0 = (ti == tj && cb > rb) ? -1 : (int)cb; f.c1 = -1; f.ke0 = 128; f.ke1 = 0;
        inc = U / NPF_UPD;
        out = acnt + ti * T + tj;
      }
      run_fine(f);
    } else {
      inc = U / NP;
      Strip st;
      st.C2 = nullptr;
      st.ldc2 = 0;
      st.active = 1;
      const int64_t R = 128 * (int64_t)ti, q = 32 * part, wv = 32 * wave;
      switch (type) {
        case 1: {  // TRSM(i, k): row strip q of L_ik = A_ik · X_kkᵀ, columns wv..
          const int64_t K = 128 * (int64_t)tk;
          st.A = p.A + (R + q) * lda + K; st.lda = lda;
          st.B = p.Linv + (K + wv) * ldl + K; st.ldb = ldl; st.bt = 1;
          st.C = p.A + (R + q) * lda + K + wv; st.ldc = lda;
          if (p.Lout) { st.C2 = p.Lout + (R + q) * p.ldlo + K + wv; st.ldc2 = p.ldlo; }
          st.alpha = 1.0; st.beta = 0.0; st.kb = 0; st.ke = (int)wv + 32;
          out = acnt + ti * T + tk;
          break;
        }
        case 2: {  // UPD(i, j, k): row strip q of A_ij −= L_ik L_jkᵀ (diagonal: lower blocks)
          const int64_t J = 128 * (int64_t)tj, K = 128 * (int64_t)tk;
          st.A = p.A + (R + q) * lda + K; st.lda = lda;
          st.B = p.A + (J + wv) * lda + K; st.ldb = lda; st.bt = 1;
          st.C = p.A + (R + q) * lda + J + wv; st.ldc = lda;
          st.alpha = -1.0; st.beta = 1.0; st.kb = 0; st.ke = 128;
          st.active = !(ti == tj && wave > part);
          out = acnt + ti * T + tj;
          break;
        }
        case 3: {  // UPDX(i, k, j): row strip q of S_ik (+)= L_ij X_jk (X_kk lower: k' >= col)
          const int64_t J = 128 * (int64_t)tj, K = 128 * (int64_t)tk;
          st.A = p.A + (R + q) * lda + J; st.lda = lda;
          st.B = p.Linv + J * ldl + K + wv; st.ldb = ldl; st.bt = 0;
          st.C = p.Linv + (R + q) * ldl + K + wv; st.ldc = ldl;
          st.alpha = 1.0; st.beta = tj == tk ? 0.0 : 1.0;
          st.kb = tj == tk ? (int)wv : 0; st.ke = 128;
          out = xcnt + ti * T + tk;
          break;
        }
        default: {  // FIN(i, k): column strip q of X_ik = −X_ii S_ik, rows wv.. (X_ii lower)
          const int64_t K = 128 * (int64_t)tk;
          st.A = p.Linv + (R + wv) * ldl + R; st.lda = ldl;
          st.B = p.Linv + R * ldl + K + q; st.ldb = ldl; st.bt = 0;
          st.C = p.Linv + (R + wv) * ldl + K + q; st.ldc = ldl;
          st.alpha = -1.0; st.beta = 0.0; st.kb = 0; st.ke = (int)wv + 32;
          out = xcnt + ti * T + tk;
          break;
        }
      }
      run_strip<G>(st);
    }
    // ---- publish: every wave's write-through stores drained, barrier; the arrival itself is
    //      the first thing lane 0 does at the top of the next iteration
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ++ndone;
  }
  // ---- the last workgroup out zeroes this launch's counters for the next launch (no memset node
  //      ahead of a replayed sequence).  Every workgroup first adds the tasks it completed to
  //      cnt[2] and waits for its own counter atomics (the last arrival and that add have no
  //      return value; vmcnt covers them), then counts itself out.
  if (tid == 0 && ndone)
    __hip_atomic_fetch_add(p.cnt + 2, ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int e = __hip_atomic_fetch_add(p.cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh[1] = e == (int)gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(sh[1])) {
    // The run is complete only if every queue slot was executed once and each workgroup fetched
    // exactly one slot past the end: counters that were not zero at launch (the round-3 "no-op
    // replay": a head counter >= ntasks makes every workgroup leave at once and Linv / logdiag
    // unwritten) are reported as error 2 instead of passing check_info silently.
    if (tid == 0) {
      const int head_end = __hip_atomic_load(p.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int done = __hip_atomic_load(p.cnt + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e == 0x7f7f7f7f && (done != p.ntasks || head_end != p.ntasks + (int)gridDim.x))
        __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int n = 16 + 2 * T * T;
    for (int i = tid; i < n; i += 256)
      __hip_atomic_store(p.cnt + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
}  // namespace dag

hipError_t launch_potrf_dag(const DagParams& p, int nwg, hipStream_t s) {
  if ((p.lda & 1) || (p.ldl & 1) || (p.Lout && (p.ldlo & 1)) || p.T < 1 || p.T > 64 || nwg < 1 ||
      !p.tasks || !p.cnt || p.ntasks < 1)
    return hipErrorInvalidValue;
  // every strip's buffer descriptor spans at most 128 rows of its matrix (32-bit offsets)
  if ((int64_t)128 * std::max(p.lda, p.ldl) * 8 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  auto k = p.trace ? (p.group == 2 ? dag::potrf_dag_kernel<true, 2>
                                    : p.group == 3 ? dag::potrf_dag_kernel<true, 3> : dag::potrf_dag_kernel<true, 4>)
                   : (p.group == 2 ? dag::potrf_dag_kernel<false, 2>
                                    : p.group == 3 ? dag::potrf_dag_kernel<false, 3> : dag::potrf_dag_kernel<false, 4>);
  if (p.group < 2 || p.group > 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k, dim3(nwg), dim3(256), 0, s, p);
  return hipGetLastError();
}

// Queue order of the persistent factorisation's tasks for a block of T tiles: tile tasks with
// their dependencies, then Kahn's algorithm releasing the ready task of best priority first (so
// the order is topological whatever the priorities), each tile task expanded into its NP strips.
//   order 0: earliest estimated start first (a forward critical-path pass; estimated µs: leaf 36,
//            strip task 4, hand-off 3) — round 3's first build;
//   order 1: largest upward rank first (the longest estimated path from the task to the end of
//            the block, with per-type durations), so the updates that feed the next leaves
//            overtake the bulk of the trailing update (the first leaves waited 20-26 µs behind
//            it), with the durations the round-4 traces measured (below);
//   order 2: the same with round 3's weights (leaf 38, strip 9, fine part 4, hand-off 1).
// fine: the leaf chain's TRSM(k+1,k) and UPD(k+1,k+1,k) as fine parts (8 / 16, see run_fine).
// (Round 4's split chain — the leaf without its inverse, TRSM(k+1,k) by substitution, an INV task
// off the chain — measured slower and was removed: profiles/r4_dag_split_ab.txt,
// profiles/r5_prune_split_chain.diff.)
// Word: type | part << 3 | fine << 7 | i << 8 | j << 16 | k << 24.
// order 1's weights, µs: LEAF, fine part, TRSM, UPD, UPDX, FIN strips, hand-off (tools/dag_bench
// overrides them for sweeps; the library never writes them)
double g_dag_weights[7] = {35.0, 6.0, 9.7, 11.7, 11.2, 9.3, 2.5};

std::vector<uint32_t> dag_task_list(int T, int order, bool fine) {
  struct Task { int type, i, j, k; std::vector<int> deps; double est = 0.0, rank = 0.0; };
  auto is_fine = [&](const Task& t) {
    return fine && ((t.type == 1 && t.i == t.k + 1) || (t.type == 2 && t.i == t.k + 1 && t.j == t.i));
  };
  std::vector<Task> tk;
  std::vector<int> leaf(T), xkk(T), trsm(T * T, -1), fin(T * T, -1);
  std::vector<int> upd_last(T * T, -1), updx_last(T * T, -1);
  auto add = [&](int type, int i, int j, int k, std::vector<int> deps) {
    Task t;
    t.type = type; t.i = i; t.j = j; t.k = k;
    for (int d : deps)
      if (d >= 0) t.deps.push_back(d);
    tk.push_back(t);
    return (int)tk.size() - 1;
  };
  // factorisation, right-looking (generation order is topological)
  for (int k = 0; k < T; ++k) {
    leaf[k] = add(0, k, k, k, {upd_last[k * T + k]});
    xkk[k] = leaf[k];  // the task X_kk comes from
    for (int i = k + 1; i < T; ++i) trsm[i * T + k] = add(1, i, k, k, {upd_last[i * T + k], xkk[k]});
    for (int j = k + 1; j < T; ++j)
      for (int i = j; i < T; ++i)
        upd_last[i * T + j] = add(2, i, j, k, {trsm[i * T + k], trsm[j * T + k], upd_last[i * T + j]});
  }
  // inverse: X row j final → its terms pushed into every row i > j
  auto xfinal = [&](int j, int k) { return j == k ? xkk[k] : fin[j * T + k]; };
  for (int j = 0; j < T; ++j) {
    for (int k = 0; k < j; ++k)  // X_jk = −X_jj S_jk once every term j' < j is in
      fin[j * T + k] = add(4, j, k, k, {updx_last[j * T + k], xkk[j]});
    for (int i = j + 1; i < T; ++i)
      for (int k = 0; k <= j; ++k)
        updx_last[i * T + k] = add(3, i, j, k, {trsm[i * T + j], xfinal(j, k), updx_last[i * T + k]});
  }
  const int n = (int)tk.size();
  std::vector<std::vector<int>> succ(n);
  std::vector<int> indeg(n, 0);
  for (int t = 0; t < n; ++t)
    for (int d : tk[t].deps) { succ[d].push_back(t); ++indeg[t]; }
  if (order == 0) {
    auto dur = [&](const Task& t) { return t.type == 0 ? 36.0 : 4.0; };
    for (int t = 0; t < n; ++t)  // generation order is topological
      for (int d : tk[t].deps) tk[t].est = std::max(tk[t].est, tk[d].est + dur(tk[d]) + 3.0);
  } else if (order == 2) {  // round 3's weights
    auto dur = [&](const Task& t) {
      return t.type == 0 ? 38.0 : is_fine(t) ? 4.0 : 9.0;
    };
    for (int t = n - 1; t >= 0; --t) {
      double m = 0.0;
      for (int s2 : succ[t]) m = std::max(m, tk[s2].rank + 1.0);
      tk[t].rank = dur(tk[t]) + m;
      tk[t].est = -tk[t].rank;
    }
  } else {
    // run time per strip task as the round-4 trace measured it (profiles/r4_dag_trace20_*.txt);
    // the fine parts count 6 (they run 8.5 but 8-16 of them in parallel) and each hand-off 2.5
    // (profiles/r4_dag_order_ab.txt: 3.6 % off the block against the round-3 weights)
    const double* w = g_dag_weights;
    auto dur = [&](const Task& t) {
      if (is_fine(t)) return w[1];
      switch (t.type) {
        case 0: return w[0];
        case 1: return w[2];
        case 2: return w[3];
        case 3: return w[4];
        default: return w[5];
      }
    };
    for (int t = n - 1; t >= 0; --t) {  // reverse generation order: successors first
      double m = 0.0;
      for (int s2 : succ[t]) m = std::max(m, tk[s2].rank + w[6]);
      tk[t].rank = dur(tk[t]) + m;
      tk[t].est = -tk[t].rank;  // smallest key first
    }
  }
  std::priority_queue<std::pair<double, int>, std::vector<std::pair<double, int>>,
                      std::greater<std::pair<double, int>>> ready;
  for (int t = 0; t < n; ++t)
    if (!indeg[t]) ready.push({tk[t].est, t});
  std::vector<uint32_t> out;
  while (!ready.empty()) {
    const int t = ready.top().second;
    ready.pop();
    const Task& x = tk[t];
    const bool f = is_fine(x);
    const int parts = x.type == 0 ? 1 : !f ? dag::NP : x.type == 1 ? dag::NPF_TRSM : dag::NPF_UPD;
    for (int q = 0; q < parts; ++q)
      out.push_back((uint32_t)x.type | (uint32_t)q << 3 | (uint32_t)f << 7 | (uint32_t)x.i << 8 |
                    (uint32_t)x.j << 16 | (uint32_t)x.k << 24);
    for (int s2 : succ[t])
      if (!--indeg[s2]) ready.push({tk[s2].est, s2});
  }
  return out;
}

hipError_t launch_potrf_leaf(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                             int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                             hipStream_t s) {
  if ((lda & 1) || (ldl & 1) || (Lout && (ldlo & 1))) return hipErrorInvalidValue;
  hipLaunchKernelGGL(v4::potrf_leaf_v4_kernel, dim3(1), dim3(256), 0, s, A, lda, Linv, ldl, Lout,
                     ldlo, logdiag, info, base, nreal);
  return hipGetLastError();
}

}  // namespace gps
