// Fused ARD / RBF Gram build for gfx950 (replaces ARD KF:7-23 and rbf SD:8-21).
//
//   out[i][j] = sf2 * exp(-0.5 * sum_k ((x_ik - x'_jk) / l_k)^2)  (+ diag_add if i == j)
//
// The reference builds this from ~5 eager n×m temporaries (mm, two bmm, subtract,
// scale, exp).  Here one pass writes each fp64 output exactly once: the kernel is
// bound by HBM write bandwidth (8 B per element; roofline "hbm").
//
// Tile: 32 rows × 128 columns per 256-thread workgroup.  Each lane owns two
// adjacent columns (one 16-byte store per row), each wave walks 8 rows.  The
// scaled features of the tile's 128 columns live in LDS transposed [k][col] so a
// lane reads its two columns with one conflict-free ds_read_b128 per feature;
// the row features are broadcast reads.  With `lower`, tiles strictly above the
// diagonal are skipped and elements with j > i are not written (the Cholesky
// reads only the lower triangle).  Rows >= n / columns >= m are padding: they
// get 0, or 1 on the diagonal when pad_identity is set, so the padded SPD
// matrix is diag(A, I) and its factor/inverse are diag(L, I) / diag(L⁻¹, I).
#include <atomic>

#include "gps_internal.h"

#include <type_traits>

namespace gps {

constexpr int kGramDevs = 64;  // devices the persistent Gram grid-size cache covers

// 16-byte non-temporal store of an output pair (each element is written once and next read by
// another launch): C3 K_ff 0.387 -> 0.36 ms against plain stores (profiles/r4_gram_ab.txt)
__device__ __forceinline__ void st_nt2(double* dst, double v0, double v1) {
  typedef double nv2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store((nv2){v0, v1}, reinterpret_cast<nv2*>(dst));
}

constexpr int GR_ROWS = 32;
constexpr int GR_COLS = 128;

template <int D>
__global__ __launch_bounds__(256) void gram_kernel(GramParams p) {
  __shared__ __attribute__((aligned(16))) double xs_col[(D ? D : GPS_MAX_D) * GR_COLS];
  __shared__ double xs_row[GR_ROWS * (D ? D : GPS_MAX_D)];
  __shared__ double2 etab[64];
  const int d = D ? D : p.d;
  const int tiles_x = p.N / GR_COLS;
  const int bx = blockIdx.x % tiles_x;
  const int by = blockIdx.x / tiles_x;
  const int c0 = bx * GR_COLS, r0 = by * GR_ROWS;
  if (p.lower && c0 > r0 + GR_ROWS - 1) return;
  const int tid = threadIdx.x;

  for (int e = tid; e < GR_COLS * d; e += 256) {
    const int j = e / d, k = e - j * d;
    const int gj = c0 + j;
    xs_col[k * GR_COLS + j] = gj < p.m ? p.xp[(int64_t)gj * d + k] * p.inv_ell[k] : 0.0;
  }
  for (int e = tid; e < GR_ROWS * d; e += 256) {
    const int i = e / d, k = e - i * d;
    const int gi = r0 + i;
    xs_row[i * d + k] = gi < p.n ? p.x[(int64_t)gi * d + k] * p.inv_ell[k] : 0.0;
  }
  exp_tab_stage(etab);
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int jl = 2 * lane;
  const int gj = c0 + jl;
  const bool colpad0 = gj >= p.m, colpad1 = gj + 1 >= p.m;

#pragma unroll 2
  for (int rr = wave; rr < GR_ROWS; rr += 4) {
    const int gi = r0 + rr;
    double a0 = 0.0, a1 = 0.0;
    if constexpr (D > 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double xr = xs_row[rr * D + k];
        const double2 xc = *reinterpret_cast<const double2*>(&xs_col[k * GR_COLS + jl]);
        const double e0 = xr - xc.x, e1 = xr - xc.y;
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
      }
    } else {
      for (int k = 0; k < d; ++k) {
        const double xr = xs_row[rr * d + k];
        const double2 xc = *reinterpret_cast<const double2*>(&xs_col[k * GR_COLS + jl]);
        const double e0 = xr - xc.x, e1 = xr - xc.y;
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
      }
    }
    double v0 = p.sf2 * exp_neg(-0.5 * a0, etab);
    double v1 = p.sf2 * exp_neg(-0.5 * a1, etab);
    const bool rowpad = gi >= p.n;
    if (gi == gj) v0 += p.diag_add;
    if (gi == gj + 1) v1 += p.diag_add;
    if (rowpad || colpad0) v0 = (p.pad_identity && gi == gj) ? 1.0 : 0.0;
    if (rowpad || colpad1) v1 = (p.pad_identity && gi == gj + 1) ? 1.0 : 0.0;
    double* dst = p.out + (int64_t)gi * p.ldo + gj;
    if (!p.lower || gj + 1 <= gi) {
      st_nt2(dst, v0, v1);
    } else if (gj <= gi) {
      dst[0] = v0;
    }
  }
}

// Register-resident variant for the compiled feature counts d = 1, 8 (16: gram_col_kernel): a 128×128
// tile per workgroup, each lane holds its two columns' scaled features in VGPRs for the
// whole tile and the 128 rows' scaled features sit in LDS, read as wave-uniform
// (broadcast) 16-byte loads.  Per element that is 2d VALU ops + exp and no per-element
// LDS traffic — gram_kernel above spends one ds_read_b128 per lane per feature per row
// on the columns, which made it LDS-issue-bound at d = 16 (C5 Knm: 2.0 TB/s).  Same
// arithmetic in the same order as gram_kernel: bitwise-identical output.
constexpr int G2_ROWS = 128;

// The d = 16 build in two launches: gram_col_kernel takes every tile but the diagonal ones when
// something happens on i == j (a diagonal add, the identity padding, the lower mask) — those few
// (one per tile row, Kmm / a lower K_ff only) go to gram_reg_kernel<16> over a compact grid.
__host__ __device__ inline bool gram_diag_special(const GramParams& p) {
  return p.diag_add != 0.0 || p.pad_identity || p.lower;
}
__host__ __device__ inline int64_t gram_edge_count(const GramParams& p) {
  const int tx = p.N / GR_COLS, ty = (p.M + G2_ROWS - 1) / G2_ROWS;
  return gram_diag_special(p) ? (tx < ty ? tx : ty) : 0;
}

template <int D>
__global__ __launch_bounds__(256) void gram_reg_kernel(GramParams p) {
  __shared__ __attribute__((aligned(16))) double xs_row[G2_ROWS * D];
  __shared__ double2 etab[64];
  const int tiles_x = p.N / GR_COLS;
  int bx = blockIdx.x % tiles_x;
  int by = blockIdx.x / tiles_x;
  if constexpr (D == 16) {  // (only the d = 16 build has an edge launch: the diagonal tiles)
    if (p.edge) bx = by = blockIdx.x;
  }
  const int c0 = bx * GR_COLS, r0 = by * G2_ROWS;
  if (p.lower && c0 > r0 + G2_ROWS - 1) return;
  const int rows = min(G2_ROWS, p.M - r0);
  const int tid = threadIdx.x;
  for (int e = tid; e < rows * D; e += 256) {
    const int i = e / D, k = e - i * D;
    const int gi = r0 + i;
    xs_row[e] = gi < p.n ? p.x[(int64_t)gi * D + k] * p.inv_ell[k] : 0.0;
  }
  const int lane = tid & 63, wave = tid >> 6;
  const int gj = c0 + 2 * lane;
  const bool colpad0 = gj >= p.m, colpad1 = gj + 1 >= p.m;
  double f0[D], f1[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    f0[k] = colpad0 ? 0.0 : p.xp[(int64_t)gj * D + k] * p.inv_ell[k];
    f1[k] = colpad1 ? 0.0 : p.xp[(int64_t)(gj + 1) * D + k] * p.inv_ell[k];
  }
  exp_tab_stage(etab);
  __syncthreads();

  // squared scaled distances of row rr to this lane's two columns
  auto dist2 = [&](int rr, double& a0, double& a1) {
    a0 = 0.0;
    a1 = 0.0;
    if constexpr (D % 2 == 0) {
#pragma unroll
      for (int k = 0; k < D; k += 2) {
        const double2 xr = *reinterpret_cast<const double2*>(&xs_row[rr * D + k]);
        double e0 = xr.x - f0[k], e1 = xr.x - f1[k];
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
        e0 = xr.y - f0[k + 1];
        e1 = xr.y - f1[k + 1];
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
      }
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double xr = xs_row[rr * D + k];
        const double e0 = xr - f0[k], e1 = xr - f1[k];
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
      }
    }
  };

  // interior tile (no padded row or column, every column index below every row index or,
  // for a full Gram, the index ranges disjoint): no diagonal add, pad or lower-mask select
  // can apply, so the per-element selects drop out of the loop.  Same values bitwise.
  const bool plain = r0 + rows <= p.n && c0 + GR_COLS <= p.m &&
                     (c0 + GR_COLS <= r0 || (!p.lower && r0 + rows <= c0));
  if (plain) {
#pragma unroll 2
    for (int rr = wave; rr < rows; rr += 4) {
      double a0, a1;
      dist2(rr, a0, a1);
      double* dst = p.out + (int64_t)(r0 + rr) * p.ldo + gj;
      st_nt2(dst, p.sf2 * exp_neg(-0.5 * a0, etab), p.sf2 * exp_neg(-0.5 * a1, etab));
    }
    return;
  }

#pragma unroll 2
  for (int rr = wave; rr < rows; rr += 4) {
    const int gi = r0 + rr;
    double a0, a1;
    dist2(rr, a0, a1);
    double v0 = p.sf2 * exp_neg(-0.5 * a0, etab);
    double v1 = p.sf2 * exp_neg(-0.5 * a1, etab);
    const bool rowpad = gi >= p.n;
    if (gi == gj) v0 += p.diag_add;
    if (gi == gj + 1) v1 += p.diag_add;
    if (rowpad || colpad0) v0 = (p.pad_identity && gi == gj) ? 1.0 : 0.0;
    if (rowpad || colpad1) v1 = (p.pad_identity && gi == gj + 1) ? 1.0 : 0.0;
    double* dst = p.out + (int64_t)gi * p.ldo + gj;
    if (!p.lower || gj + 1 <= gi) {
      st_nt2(dst, v0, v1);
    } else if (gj <= gi) {
      dst[0] = v0;
    }
  }
}

// d = 16: the same 128×128 tile with ONE column per lane — waves 0 / 1 own columns 0-63 / 64-127
// of the even rows, waves 2 / 3 of the odd rows — so a lane holds 16 features instead of 32 (60
// VGPRs instead of 122: 8 waves per SIMD instead of 4) and stores 8 bytes per row.  Padded rows
// and columns are zero-filled here; the diagonal tiles of a build with a diagonal add, identity
// padding or the lower mask (Kmm, a lower K_ff) go to gram_reg_kernel<16> in a second launch of
// one workgroup per tile row (with those selects in this kernel it needed 78 VGPRs, or spilled at
// 64, and a kernel with scratch ran slower everywhere).  C5-shaped Knm (100096 × 4096) 2.85 →
// 3.34 TB/s (profiles/r5i_gram_cols.txt; at d = 8 the two-column kernel is as fast).  Same
// arithmetic in the same order: bitwise-identical output.
template <int D>
__global__ __launch_bounds__(256) void gram_col_kernel(GramParams p) {
  __shared__ __attribute__((aligned(16))) double xs_row[G2_ROWS * D];
  __shared__ double2 etab[64];
  const int tiles_x = p.N / GR_COLS;
  const int bx = blockIdx.x % tiles_x;
  const int by = blockIdx.x / tiles_x;
  if ((p.lower && bx > by) || (bx == by && gram_diag_special(p))) return;
  const int c0 = bx * GR_COLS, r0 = by * G2_ROWS;
  const int rows = min(G2_ROWS, p.M - r0);
  const int tid = threadIdx.x;
  for (int e = tid; e < rows * D; e += 256) {
    const int i = e / D, k = e - i * D;
    const int gi = r0 + i;
    xs_row[e] = gi < p.n ? p.x[(int64_t)gi * D + k] * p.inv_ell[k] : 0.0;
  }
  const int gj = c0 + (tid & (GR_COLS - 1)), half = tid >> 7;
  const bool colpad = gj >= p.m;
  double f[D];
#pragma unroll
  for (int k = 0; k < D; ++k)  // (a padded column reads the last real one; its outputs are 0)
    f[k] = p.xp[(int64_t)(colpad ? p.m - 1 : gj) * D + k] * p.inv_ell[k];
  exp_tab_stage(etab);
  __syncthreads();
  const int rend = min(rows, p.n - r0);  // real rows of the tile; the padded ones below get 0
#pragma unroll 2
  for (int rr = half; rr < rend; rr += 2) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < D; k += 2) {
      const double2 xr = *reinterpret_cast<const double2*>(&xs_row[rr * D + k]);
      double e = xr.x - f[k];
      a = fma(e, e, a);
      e = xr.y - f[k + 1];
      a = fma(e, e, a);
    }
    const double v = p.sf2 * exp_neg(-0.5 * a, etab);
    __builtin_nontemporal_store(colpad ? 0.0 : v, p.out + (int64_t)(r0 + rr) * p.ldo + gj);
  }
  for (int rr = max(rend, 0) + ((max(rend, 0) & 1) != half ? 1 : 0); rr < rows; rr += 2)
    p.out[(int64_t)(r0 + rr) * p.ldo + gj] = 0.0;
}

// d = 8 / 16 builds on the matrix cores, in the reference's own form (ARD KF:15-22:
// res = 2·x·x'ᵀ − ‖x‖² − ‖x'‖², then sf2·exp(½·res)): per 16×16 output block d/4
// v_mfma_f64_16x16x4 for the cross products and ~20 VALU ops per element (two subtractions,
// the exp, the scale) instead of the direct difference's 2d + 20 — at d = 16 the direct form is
// VALU-bound (C5 Knm 3.9 TB/s).  Output differs from the direct-difference kernels by rounding
// only: |Δres| ≲ ε·(‖x − c‖² + ‖x' − c‖²), with both sides shifted by the same point c — the
// scaled features of the row tile's first row — so that an offset in the data (the reference's
// uncentred expansion loses ε·‖x‖²) costs no more than in the direct difference.
//
// Persistent: the grid is sized to the chip and workgroup b takes the items (128×128 tiles,
// row-major; with `lower` the tiles on or below the diagonal of a square build) either as the
// contiguous run [b·T/G, (b+1)·T/G) (S = false: the row features' MFMA fragments and half norms
// are staged once per row tile) or strided b, b + G, ... (S: the workgroups resident at one time
// write neighbouring tiles, each item restages its rows); either way the next item's features
// are in flight (registers) while the current one computes.
// The scaled features of the tile's rows / columns sit in LDS with row stride d + 1 doubles (the
// 16 rows a fragment read touches fall in distinct banks); thread t stages half a feature row
// (row t/2, features (t&1)·d/2..) and the lane pair completes the row's squared norm.  Wave w
// owns rows 32w..32w+31 of a tile and walks its 8 column blocks; each lane stores 4 rows × 1
// column per block (the accumulator layout: 4 × 128 contiguous bytes per store instruction).
// Diagonal tiles of a build with a diagonal add / identity padding / the lower mask, and tiles
// with padded rows or columns, take the per-element selects; every other tile skips them.
template <int D>
__device__ __forceinline__ void gram_stage_half(const double* __restrict__ src, int rows_real,
                                                int base, const double* inv_ell,
                                                const double* __restrict__ cen, double (&v)[D / 2]) {
  const int t = threadIdx.x, gi = base + (t >> 1), k0 = (t & 1) * (D / 2);
#pragma unroll
  for (int k = 0; k < D / 2; ++k) {
    // (a non-finite centre coordinate is replaced by 0 — the same shift for both sides, so
    //  still exact — lest one bad input row poison its whole tile instead of its own row)
    const double c = cen[k0 + k] * inv_ell[k0 + k];
    v[k] = gi < rows_real ? src[(int64_t)gi * D + k0 + k] * inv_ell[k0 + k] - (isfinite(c) ? c : 0.0)
                          : 0.0;
  }
}
template <int D>
__device__ __forceinline__ void gram_put_half(double* xs, double* hs, const double (&v)[D / 2]) {
  constexpr int LS = D + 1;
  const int t = threadIdx.x, r = t >> 1, k0 = (t & 1) * (D / 2);
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < D / 2; ++k) {
    xs[r * LS + k0 + k] = v[k];
    s = fma(v[k], v[k], s);
  }
  s += __shfl_xor(s, 1);
  if (!(t & 1)) hs[r] = 0.5 * s;  // ½‖x‖²: res/2 = x·x' − ½‖x‖² − ½‖x'‖², the same rounding
}
// item -> (row tile, column tile); lower: the lower-triangular tiles of a square build, row-major
__device__ __forceinline__ void gram_item(int64_t it, int tiles_x, bool lower, int& by, int& bx) {
  if (lower) {
    int r = (int)((sqrt(8.0 * (double)it + 1.0) - 1.0) * 0.5);
    while ((int64_t)r * (r + 1) / 2 > it) --r;
    while ((int64_t)(r + 1) * (r + 2) / 2 <= it) ++r;
    by = r;
    bx = (int)(it - (int64_t)r * (r + 1) / 2);
  } else {
    by = (int)(it / tiles_x);
    bx = (int)(it - (int64_t)by * tiles_x);
  }
}

template <int D, bool S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gram_mfma_kernel(GramParams p) {
  static_assert(D % 8 == 0, "k-steps of 4, half rows");
  constexpr int LS = D + 1;
  __shared__ double xr[G2_ROWS * LS];
  __shared__ double xc[GR_COLS * LS];
  __shared__ double hr[G2_ROWS], hc[GR_COLS];
  __shared__ double2 etab[64];
  const int tiles_x = p.N / GR_COLS, tiles_m = (p.M + G2_ROWS - 1) / G2_ROWS;
  const int64_t T = p.lower ? (int64_t)tiles_m * (tiles_m + 1) / 2 : (int64_t)tiles_m * tiles_x;
  // S: items blockIdx.x, + gridDim.x, ... (the workgroups resident at one time write neighbouring
  // tiles); otherwise the contiguous run [b·T/G, (b+1)·T/G)
  const int64_t step = S ? gridDim.x : 1;
  const int64_t end = S ? T : (int64_t)(blockIdx.x + 1) * T / gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const bool special = gram_diag_special(p);
  exp_tab_stage(etab);
  typedef double d4v __attribute__((ext_vector_type(4)));
  double a[2][D / 4], pv[D / 2], qv[S ? D / 2 : 1];
  int cur_by = -1, by, bx;
  int64_t it = S ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * T / gridDim.x;
  auto stage_next = [&](int nby, int nbx) {  // the item's column (and with S its row) features
    const double* cen = p.x + (int64_t)min(nby * G2_ROWS, p.n - 1) * D;
    gram_stage_half<D>(p.xp, p.m, nbx * GR_COLS, p.inv_ell, cen, pv);
    if constexpr (S) gram_stage_half<D>(p.x, p.n, nby * G2_ROWS, p.inv_ell, cen, qv);
  };
  if (it < end) {
    gram_item(it, tiles_x, p.lower, by, bx);
    stage_next(by, bx);
  }
  for (; it < end; it += step) {
    gram_item(it, tiles_x, p.lower, by, bx);
    const int c0 = bx * GR_COLS, r0 = by * G2_ROWS;
    const int rows = min(G2_ROWS, p.M - r0);  // a multiple of 32 (launch_gram checks M % 32)
    __syncthreads();  // the previous tile's reads of xc / hc / xr are done
    if (by != cur_by) {
      if constexpr (S) {
        gram_put_half<D>(xr, hr, qv);
      } else {
        double rv[D / 2];
        gram_stage_half<D>(p.x, p.n, r0, p.inv_ell, p.x + (int64_t)min(r0, p.n - 1) * D, rv);
        gram_put_half<D>(xr, hr, rv);
      }
    }
    gram_put_half<D>(xc, hc, pv);
    __syncthreads();
    if (by != cur_by) {
      cur_by = by;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int rt = 32 * wave + 16 * rb;
#pragma unroll
        for (int kk = 0; kk < D / 4; ++kk) a[rb][kk] = xr[(rt + lr) * LS + 4 * kk + lg];
      }
    }
    if (it + step < end) {  // the next item's features, in flight while this one computes
      int nby, nbx;
      gram_item(it + step, tiles_x, p.lower, nby, nbx);
      stage_next(nby, nbx);
    }
    if (32 * wave >= rows) continue;
    const bool plain = r0 + rows <= p.n && c0 + GR_COLS <= p.m && !(bx == by && special);
    const int rw = r0 + 32 * wave;
    double* const obase = p.out + (int64_t)rw * p.ldo + c0;
    // one column block of 16, row block rb: the cross products, then the elements
    // (PLAIN: no selects; the edge tiles walk their row blocks one at a time, which keeps their
    // selects within the plain path's registers)
    auto rowblock = [&](int cb, int rb, const double (&b)[D / 4], double hcol, auto plain_tag) {
      constexpr bool PLAIN = decltype(plain_tag)::value;
      const int gj = c0 + 16 * cb + lr;
      d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < D / 4; ++kk)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[rb][kk], b[kk], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = 16 * rb + 4 * q + lg;
        double v = p.sf2 * exp_neg((acc[q] - hr[32 * wave + rl]) - hcol, etab);
        double* dst = obase + (int64_t)rl * p.ldo + 16 * cb + lr;
        if constexpr (PLAIN) {
          __builtin_nontemporal_store(v, dst);
        } else {
          const int gi = rw + rl;
          if (gi == gj) v += p.diag_add;
          if (gi >= p.n || gj >= p.m) v = (p.pad_identity && gi == gj) ? 1.0 : 0.0;
          if (!p.lower || gj <= gi) __builtin_nontemporal_store(v, dst);
        }
      }
    };
    auto block = [&](int cb, auto plain_tag) {
      constexpr bool PLAIN = decltype(plain_tag)::value;
      double b[D / 4];
#pragma unroll
      for (int kk = 0; kk < D / 4; ++kk) b[kk] = xc[(16 * cb + lr) * LS + 4 * kk + lg];
      const double hcol = hc[16 * cb + lr];
      if constexpr (PLAIN) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) rowblock(cb, rb, b, hcol, plain_tag);
      } else {
#pragma unroll 1
        for (int rb = 0; rb < 2; ++rb) rowblock(cb, rb, b, hcol, plain_tag);
      }
    };
    if (plain) {
#pragma unroll 1
      for (int cb = 0; cb < GR_COLS / 16; ++cb) block(cb, std::true_type{});
    } else {
#pragma unroll 1
      for (int cb = 0; cb < GR_COLS / 16; ++cb) block(cb, std::false_type{});
    }
  }
}

// GPS_OPT_GRAM_REG (process-wide): 0 = the LDS-column kernel for every d; 1 = the register-
// resident direct-difference kernels for d in {1, 8, 16} (bitwise equal to 0); 2 (default) = as
// 1 with the d = 8 and 16 builds on the matrix-core kernel (C3 K_ff 0.383 -> 0.351 ms, K*f
// 0.220 -> 0.192, C5 Knm 1.70 -> 1.47: profiles/r5am_gram_ab.json)
int g_gram_reg = 2;

hipError_t launch_gram(const GramParams& p, hipStream_t s) {
  if (p.d < 1 || p.d > GPS_MAX_D || p.M % GR_ROWS || p.N % GR_COLS || (p.ldo & 1))
    return hipErrorInvalidValue;
  if (g_gram_reg == 2 && (p.d == 8 || p.d == 16) && (!p.lower || p.M == p.N)) {
    const int64_t tm = (p.M + G2_ROWS - 1) / G2_ROWS, tx = p.N / GR_COLS;
    const int64_t items = p.lower ? tm * (tm + 1) / 2 : tm * tx;
    if (items == 0) return hipSuccess;
    // d = 16 walks contiguous runs of tiles (row fragments staged once per row tile), d = 8
    // strided items (the resident workgroups write neighbouring tiles; its staging is half as
    // large): C5 Knm 1.47 vs 1.87 ms, C3 K_ff 0.351 vs 0.390 and K*f 0.192 vs 0.225 ms the
    // other way round (profiles/r5am_gram_ab.json, mode 2 = contiguous at both, 3 = strided)
    const void* fn = p.d == 8 ? (const void*)gram_mfma_kernel<8, true> : (const void*)gram_mfma_kernel<16, false>;
    // persistent over one resident wave of the grid (as many workgroups as fit on every CU at
    // once); a build of fewer than 4 such waves of tiles runs one tile per workgroup instead
    // (2-3 tiles per workgroup would leave the last round a third full: C5 K*m)
    // (cached per device and d: host threads driving contexts on different devices launch
    //  concurrently — ADVICE r5 — so the cache is atomic and keyed by the current device)
    static std::atomic<int> slots[kGramDevs][2];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kGramDevs) return hipErrorInvalidValue;
    int sl = slots[dev][p.d == 16].load(std::memory_order_relaxed);
    if (!sl) {
      int cus = 0, per = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0) != hipSuccess || cus < 1 ||
          per < 1)
        return hipErrorInvalidValue;
      sl = cus * per;
      slots[dev][p.d == 16].store(sl, std::memory_order_relaxed);
    }
    const int64_t g = items < 4 * (int64_t)sl ? items : sl;
    GramParams q = p;
    void* args[] = {&q};
    return hipLaunchKernel(fn, dim3((unsigned)g), dim3(256), args, 0, s);
  }
  if (g_gram_reg && (p.d == 1 || p.d == 8 || p.d == 16)) {
    const int64_t blocks = (int64_t)((p.M + G2_ROWS - 1) / G2_ROWS) * (p.N / GR_COLS);
    if (blocks == 0) return hipSuccess;
    dim3 grid((unsigned)blocks), block(256);
    switch (p.d) {
      case 1: hipLaunchKernelGGL(gram_reg_kernel<1>, grid, block, 0, s, p); break;
      case 8: hipLaunchKernelGGL(gram_reg_kernel<8>, grid, block, 0, s, p); break;
      default: {
        hipLaunchKernelGGL(gram_col_kernel<16>, grid, block, 0, s, p);
        GramParams q = p;
        q.edge = 1;
        const int64_t e = gram_edge_count(p);
        if (e > 0) hipLaunchKernelGGL(gram_reg_kernel<16>, dim3((unsigned)e), block, 0, s, q);
        break;
      }
    }
    return hipGetLastError();
  }
  const int64_t blocks = (int64_t)(p.M / GR_ROWS) * (p.N / GR_COLS);
  if (blocks == 0) return hipSuccess;
  dim3 grid((unsigned)blocks), block(256);
  switch (p.d) {
    case 1: hipLaunchKernelGGL(gram_kernel<1>, grid, block, 0, s, p); break;
    case 8: hipLaunchKernelGGL(gram_kernel<8>, grid, block, 0, s, p); break;
    case 16: hipLaunchKernelGGL(gram_kernel<16>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(gram_kernel<0>, grid, block, 0, s, p); break;
  }
  return hipGetLastError();
}

}  // namespace gps
