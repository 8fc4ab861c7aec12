// EXPERIMENT (not in the library): an MFMA-tiled leaf, measured 55 µs per 128 block against
// the production kernel's 51 µs (csrc/kernels_potrf.hip) — see DESIGN.md §6.
// Leaf of the recursive Cholesky (the diagonal 128×128 block; replaces LAPACK ?potrf behind
// torch.potrf, KF:26 / KF:332) fused with the block's triangular inverse, on the FP64 MFMA.
//
// One 256-thread workgroup (4 waves) factors A = UᵀU (U = Lᵀ) in 16×16 tiles, right-looking,
// and forms L⁻¹ row-block by row-block behind the factorisation (left-looking trtri), so the
// whole 128 block is one launch.  All 36 upper tiles S_ab (a ≤ b) live in LDS in the
// v_mfma_f64_16x16x4 accumulator order (lane l = (c = l & 15, g = l >> 4), register r:
// S[4r + g][c]); loaded into registers that order is the B operand of the tile as it stands,
// and as the A operand it supplies the tile's transpose — so every product below is
// (stored)ᵀ·(stored) and nothing is re-laid-out.  Step p (8 steps):
//   A  wave 0 factors S_pp column-per-lane (lane c holds column c of the symmetric tile, the
//      four 16-lane DPP rows redundantly): 16 pivots, one rsqrt each, every broadcast of the
//      pivot column one v_mov_b64 row_newbcast; X = L_pp⁻¹ rides on the same broadcasts.
//      Waves 1-3 meanwhile form row-block p−1 of L⁻¹.
//   B  panel   U_pb = L_pp⁻¹ S_pb   (X read in the A-operand order from its row-major copy)
//   C  update  S_ab −= U_paᵀ U_pb,  p < a ≤ b
//   L⁻¹ (= Z, lower): Z_aa = X_a,  Z_ba = −X_b Σ_{k=a}^{b−1} U_kbᵀ Z_ka  (b > a).
// Every loop except the 16 pivots is a run-time loop: the code stays a few KiB and is fetched
// once (a fully unrolled register-resident form was 140 KiB of straight-line code and ran at
// instruction-fetch speed, ~0.5 B/cycle: 50 µs per leaf).
// log L_ii (the ½log|A| terms of KF:332) comes from each pivot; a non-positive (or NaN) pivot
// d_k is flagged where it is seen, so the smallest flagged index is torch.potrf's "leading
// minor of order k" (info, atomicMin).
#include "gps_internal.h"

namespace gps {

namespace leafx {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int NTL = 8;  // 16×16 tiles per edge of the 128 leaf

// index of tile (a, b), a ≤ b (0..35), and of an off-diagonal pair a < b (0..27)
__host__ __device__ constexpr int tidx(int a, int b) { return 8 * a - a * (a - 1) / 2 + (b - a); }
__host__ __device__ constexpr int pidx(int a, int b) { return 7 * a - a * (a - 1) / 2 + (b - a - 1); }

// LDS map (doubles); tile slots are 256 doubles in accumulator order [r][lane]
constexpr int T_SZ = 256;
constexpr int L_ST = 0;                  // S_ab / U_ab, a ≤ b (36 slots)
constexpr int L_Z = L_ST + 36 * T_SZ;    // Z_ba = (L⁻¹)_ba, b > a (28 slots)
constexpr int L_X = L_Z + 28 * T_SZ;     // X_p = L_pp⁻¹, row-major 16×16 (8 slots)
constexpr int L_TOTAL = L_X + 8 * T_SZ;  // 18432 doubles = 144 KiB

__device__ __forceinline__ double bcast16(double v, int k) {
  // lane k of each 16-lane row to the whole row (v_mov_b64 row_newbcast:k, gfx90a+)
  long long x = __double_as_longlong(v);
  long long r;
  switch (k) {
#define GPS_NB(K) case K: r = __builtin_amdgcn_update_dpp(0ll, x, 0x150 + K, 0xf, 0xf, false); break;
    GPS_NB(0) GPS_NB(1) GPS_NB(2) GPS_NB(3) GPS_NB(4) GPS_NB(5) GPS_NB(6) GPS_NB(7)
    GPS_NB(8) GPS_NB(9) GPS_NB(10) GPS_NB(11) GPS_NB(12) GPS_NB(13) GPS_NB(14)
    default: r = __builtin_amdgcn_update_dpp(0ll, x, 0x150 + 15, 0xf, 0xf, false); break;
#undef GPS_NB
  }
  return __longlong_as_double(r);
}

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void ld_tile(const double* sm, int base, int lane, double (&v)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = sm[base + r * 64 + lane];
}
__device__ __forceinline__ void st_tile(double* sm, int base, int lane, const d4& v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) sm[base + r * 64 + lane] = v[r];
}
// X (row-major) in the A-operand order that supplies X itself: register r = X[c][4r + g]
__device__ __forceinline__ void ld_x_as_a(const double* sm, int p, int lane, double (&v)[4]) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = sm[L_X + p * T_SZ + c * 16 + 4 * r + g];
}
// X in the B-operand order: register r = X[4r + g][c]
__device__ __forceinline__ void ld_x_as_b(const double* sm, int p, int lane, double (&v)[4]) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = sm[L_X + p * T_SZ + (4 * r + g) * 16 + c];
}

struct LeafArgs {
  const double* A; int64_t lda;
  double* Linv; int64_t ldl;
  double* Lout; int64_t ldlo;
  double* logdiag; int* info;
  int base, nreal;
};

// wave 0, step p: factor + invert the 16×16 S_pp; X row-major to LDS; outputs
__device__ __forceinline__ void leaf_pivot(double* sm, const LeafArgs& g, int lane, int p) {
  const int c = lane & 15;
  const int tb = L_ST + tidx(p, p) * T_SZ;
  double a[16], x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {  // column c of the symmetric tile: S[i][c]
    a[i] = sm[tb + (i >> 2) * 64 + (i & 3) * 16 + c];
    x[i] = i == c ? 1.0 : 0.0;
  }
  // Lane c's column is updated while c > k and left unscaled from its own pivot on (q = 0):
  // the Schur-complement column at pivot c is L_·c · L_cc, scaled by 1/L_cc at the end — no
  // per-element select in the loop.  X = L⁻¹ rides on the same broadcasts:
  // X_k· /= L_kk, X_i· −= L_ik X_k· with L_ik = w / L_kk, w = A_ik before scaling.
  double invc = 0.0, dcc = 0.0;  // 1 / L_cc and the pivot value d_c of this lane's column
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double dk = bcast16(a[k], k);
    const double inv = rsqrt(dk);                     // 1 / L_kk
    const double q = c > k ? a[k] * inv * inv : 0.0;  // L_ck / L_kk
    if (c == k) {
      invc = inv;
      dcc = dk;
    }
    const double xk = x[k] * inv;
    x[k] = xk;
    const double qx = xk * inv;
#pragma unroll
    for (int i = k + 1; i < 16; ++i) {
      const double w = bcast16(a[i], k);  // A_ik, the pivot column before its scaling
      x[i] = fma(-w, qx, x[i]);
      a[i] = fma(-w, q, a[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] *= invc;
  // lane c holds column c of L (a[i], i ≥ c) and of X = L⁻¹ (x[i], zero above c).  The pivot
  // test uses d_c as seen at its own step: a bad pivot poisons later columns AND the finished
  // ones (0·NaN), so only that value identifies the first.
  const int r0 = 16 * p;
  if (lane < 16) {
    if (!(dcc > 0.0) && r0 + c < g.nreal) atomicMin(g.info, g.base + r0 + c + 1);
    g.logdiag[r0 + c] = 0.5 * log(dcc);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      g.Linv[(int64_t)(r0 + i) * g.ldl + r0 + c] = x[i];
      sm[L_X + p * T_SZ + i * 16 + c] = x[i];
    }
    if (g.Lout) {
#pragma unroll
      for (int i = 0; i < 16; ++i) g.Lout[(int64_t)(r0 + i) * g.ldlo + r0 + c] = i >= c ? a[i] : 0.0;
    }
  }
}

// row-block b of L⁻¹: Z_ba for a < b, a ≡ (w − w0) mod nw; to LDS and to Linv
__device__ void leaf_trtri_row(double* sm, const LeafArgs& g, int lane, int w, int b, int nw,
                               int w0) {
  const int c = lane & 15, gq = lane >> 4;
  if (w < w0) return;
  double e[4];
  ld_x_as_a(sm, b, lane, e);
  for (int a = w - w0; a < b; a += nw) {
    d4 t = {0.0, 0.0, 0.0, 0.0};
    for (int k = a; k < b; ++k) {  // T += U_kbᵀ Z_ka
      double u[4], z[4];
      ld_tile(sm, L_ST + tidx(k, b) * T_SZ, lane, u);
      if (k == a) ld_x_as_b(sm, a, lane, z);
      else ld_tile(sm, L_Z + pidx(a, k) * T_SZ, lane, z);
#pragma unroll
      for (int r = 0; r < 4; ++r) t = mfma(u[r], z[r], t);
    }
    d4 zt = {0.0, 0.0, 0.0, 0.0};  // Z_ba = −X_b T
#pragma unroll
    for (int r = 0; r < 4; ++r) zt = mfma(-e[r], t[r], zt);
    st_tile(sm, L_Z + pidx(a, b) * T_SZ, lane, zt);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      g.Linv[(int64_t)(16 * b + 4 * r + gq) * g.ldl + 16 * a + c] = zt[r];
  }
}

__global__ __launch_bounds__(256) void potrf_leaf128_kernel(LeafArgs g) {
  __shared__ __attribute__((aligned(16))) double sm[L_TOTAL];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = lane & 15, gq = lane >> 4;
  // ---- S_ab = A_ab (upper tiles) from the lower-stored block
  for (int t = w; t < 36; t += 4) {
    int a = 0;
    while (tidx(a, NTL - 1) < t) ++a;
    const int b = a + t - tidx(a, a);
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * a + 4 * r + gq, j = 16 * b + c;  // element (i, j); mirrored if i < j
      v[r] = i >= j ? g.A[(int64_t)i * g.lda + j] : g.A[(int64_t)j * g.lda + i];
    }
    st_tile(sm, L_ST + t * T_SZ, lane, v);
  }
  __syncthreads();
  for (int p = 0; p < NTL; ++p) {
    // ---- A: pivot (wave 0) | row-block p−1 of L⁻¹ (waves 1-3)
    if (w == 0) leaf_pivot(sm, g, lane, p);
    else if (p >= 2) leaf_trtri_row(sm, g, lane, w, p - 1, 3, 1);
    __syncthreads();
    if (p == NTL - 1) break;
    // ---- B: panel U_pb = X_p S_pb, b = p+1+w, p+1+w+4, ...
    if (p + 1 + w < NTL) {
      double e[4];
      ld_x_as_a(sm, p, lane, e);
      for (int b = p + 1 + w; b < NTL; b += 4) {
        const int tb = L_ST + tidx(p, b) * T_SZ;
        double s[4];
        ld_tile(sm, tb, lane, s);
        d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) u = mfma(e[r], s[r], u);
        st_tile(sm, tb, lane, u);
        if (g.Lout) {  // L_bp = U_pbᵀ
#pragma unroll
          for (int r = 0; r < 4; ++r)
            g.Lout[(int64_t)(16 * b + c) * g.ldlo + 16 * p + 4 * r + gq] = u[r];
        }
      }
    }
    __syncthreads();
    // ---- C: S_ab −= U_paᵀ U_pb over the (7−p)(8−p)/2 tiles p < a ≤ b, row-major from
    // (p+1, p+1), dealt round robin (the next pivot tile goes to wave 0)
    {
      const int m = NTL - 1 - p, nt = m * (m + 1) / 2;
      for (int j = w; j < nt; j += 4) {
        int a = p + 1, rem = j;
        while (rem >= NTL - a) {
          rem -= NTL - a;
          ++a;
        }
        const int b = a + rem;
        double ua[4], ub[4], s[4];
        ld_tile(sm, L_ST + tidx(p, a) * T_SZ, lane, ua);
        ld_tile(sm, L_ST + tidx(p, b) * T_SZ, lane, ub);
        const int tb = L_ST + tidx(a, b) * T_SZ;
        ld_tile(sm, tb, lane, s);
        d4 t = {s[0], s[1], s[2], s[3]};
#pragma unroll
        for (int r = 0; r < 4; ++r) t = mfma(-ua[r], ub[r], t);
        st_tile(sm, tb, lane, t);
      }
    }
    __syncthreads();
  }
  // ---- last row-block of L⁻¹ on all four waves
  leaf_trtri_row(sm, g, lane, w, NTL - 1, 4, 0);
  // zeros above the 16-tile diagonal of Linv (and of Lout): tiles (a, b), a < b
  for (int e = threadIdx.x; e < 28 * 256; e += 256) {
    const int t = e >> 8, w16 = e & 255;
    int a = 0;
    while (pidx(a, NTL - 1) < t) ++a;
    const int b = t - pidx(a, a + 1) + a + 1;
    const int i = 16 * a + (w16 >> 4), j = 16 * b + (w16 & 15);
    g.Linv[(int64_t)i * g.ldl + j] = 0.0;
    if (g.Lout) g.Lout[(int64_t)i * g.ldlo + j] = 0.0;
  }
}

}  // namespace leafx
using namespace leafx;

hipError_t launch_potrf_leaf_mfma(const double* A, int64_t lda, double* Linv, int64_t ldl, double* Lout,
                             int64_t ldlo, double* logdiag, int* info, int base, int nreal,
                             hipStream_t s) {
  LeafArgs g{A, lda, Linv, ldl, Lout, ldlo, logdiag, info, base, nreal};
  hipLaunchKernelGGL(potrf_leaf128_kernel, dim3(1), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace gps
