// Internal declarations shared by the gfx950 kernels and the C-ABI layer.
// Everything here is float64; all device matrices are row-major and every
// dimension handed to a kernel is padded to a multiple of GPS_TILE (128).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#define GPS_TILE 128
#define GPS_MAX_D 64

namespace gps {

inline int64_t pad_to(int64_t n, int64_t t = GPS_TILE) { return (n + t - 1) / t * t; }

// ---------------------------------------------------------------- kernel params
struct GramParams {
  const double* x;    // [n][d] raw features
  const double* xp;   // [m][d]
  double* out;        // [M_pad][ldo]
  int64_t ldo;
  int n, m;           // real rows / cols
  int M, N;           // padded rows / cols written
  int d;
  double sf2;
  double diag_add;    // added where i == j (real rows)
  int lower;          // write only j <= i (tile-granular skip + element mask)
  int pad_identity;   // 1.0 on the padded diagonal (i == j >= n)
  double inv_ell[GPS_MAX_D];
  int edge;           // (launch_gram) the diagonal-tile launch of a d = 16 build (kernels_gram.hip)
};

enum Layout { LAY_N = 0, LAY_T = 1 };
// triangular structure of an operand, expressed as a k-range restriction per tile
enum Tri {
  TRI_NONE = 0,
  TRI_K_LE_I = 1,  // k < (ti+1)*128   (A lower, A[i][k] != 0 only for k <= i)
  TRI_K_LE_J = 2,  // k < (tj+1)*128   (B = Lᵀ with L lower stored [j][k])
  TRI_K_GE_J = 3,  // k >= tj*128      (B lower stored [k][j])
  TRI_K_GE_I = 4,  // k >= ti*128      (A = Lᵀ with L lower stored [k][i])
  TRI_KR_J = 5,    // k in [kr[2g], kr[2g'+1]) over the 16-column groups g..g' of the tile
                   // (B block-diagonal with unaligned blocks: block-LOO gradients)
};
enum Epi { EPI_STORE = 0, EPI_ROWSQ = 1, EPI_COLRED = 2, EPI_ROWSQ_DOT = 3 };
// EPI_ROWSQ_DOT: EPI_ROWSQ plus, in the last column tile (the full K range), out1[row] = A[row,:]·w

struct GemmParams {
  const double* A; int64_t lda;
  const double* B; int64_t ldb;
  double* C; int64_t ldc;
  int64_t c_kslice_stride;   // split-K: slice s writes C + s*stride (beta must be 0)
  int M, N, K;               // multiples of 128 (K: multiple of 16 after tri clipping)
  double alpha, beta;
  const double* kscale;      // optional per-k scale applied to A (length K)
  const double* w;           // EPI_COLRED weights (length M)
  double* out0; double* out1; int64_t ld_out;
  int lower_out;             // enumerate only tiles with tj <= ti
  int ksplit;                // number of K slices (grid.y)
  int tri;
  int tri_off;               // global index of output row / column 0 for the tri clipping (a
                             // row or column block of a larger triangular product)
  const int* kr;            // TRI_KR_J: per 16-column group [k begin, k end) (multiples of 16)
  int tiles_m, tiles_n;
  int map_mode;              // tile order: 0 auto (see tile_of), 1 grouped raster only, 2 + XCD remap,
                             // 3 XCD-banded heaviest-first (auto for triangular), 4 pre-3 auto,
                             // 5 XCD-banded 8×8 patches, 6 paired column tiles (EPI_ROWSQ*)
  int tile;                  // output tile edge: 0 auto (gemm_plan), 64 or 128
  double* ws;                // split-K workspace: slabs + ordered reduction (auto plan only
  int64_t ws_cap;            //   splits while ksplit*M*N <= ws_cap doubles)
  int* sk_cnt;               // stream-K tail (launch_gemm): per-tile arrival tickets, zero at the
                             // launch and left zero; partial tiles go to ws.  NULL: no stream-K
  int sk_slots;              // workgroup slots of the chip (2 per CU for the 128-tile kernel)
  // set by launch_gemm for the stream-K tail: tiles [sk_dp, tiles) are split over sk_wgs blocks
  int sk_dp, sk_wgs;
  int prio;                  // 1: the mainloop's MFMA phase at raised wave priority (launch_gemm)
  int mirror;                // lower_out square launch: also write the strictly-lower 32-tiles'
                             // transposes above the diagonal (a symmetric result, in the split-K
                             // reduction when there is one, else by launch_sym_mirror)
  int slab_xcd;              // set by launch_gemm (g_slab_xcd): a split-K grid's (tile, slice)
                             // pairs dealt slice-major in contiguous runs per XCD
  int kend;                  // > 0 (a multiple of 16): A's columns k >= kend are zero (the FITC row
                             // norms: kend = m rounded to 16) — the K loop stops there
  int sk_alone;              // the launch runs without a concurrent forked product (potrf_inv_rec's
                             // trailing update when nothing is forked beside it): the stream-K
                             // tail fills its last round (GPS_OPT_STREAM_K = 2, the default)
  // Row norms behind a running persistent factorisation (EPI_ROWSQ, TRI_K_LE_J, tri_off 0, 128
  // tiles, no split): column tile j needs row tile j of L⁻¹ only.
  //   dep_mode 1 (the dependent launch): each workgroup takes the heaviest column tile whose row
  //     is final (dep_sig[kSigRdy + j]) from the per-XCD queues dep_q, waiting for a row only once
  //     every workgroup of the factorisation has started (dep_sig[kSigStarted] >= dep_grid: they
  //     are resident, so the wait cannot starve them); otherwise it leaves the tile to
  //   dep_mode 2 (the completion launch, stream-ordered after the factorisation): block b is tile
  //     (b % tiles_m, tiles_n − 1 − b / tiles_m), skipped if the dependent launch took it.
  int* dep_sig; int* dep_q; int* dep_err; int dep_grid; int dep_mode;
};
// The signal block of a persistent factorisation with a dependent row-norm launch (int words,
// zeroed before the pair is launched; DagParams::sig, GemmParams::dep_sig / dep_q)
constexpr int kSigStarted = 0;   // workgroups of the factorisation that have started
constexpr int kSigRowCnt = 64;   // [64] per row tile of L⁻¹: FIN strips completed
constexpr int kSigRdy = 128;     // [64] per row tile: 1 once the row of L⁻¹ is final (2: and
                                 // every band of that column taken by the dependent launch)
constexpr int kSigQueue = 192;   // [8 XCDs][64 column tiles] queue heads of one dependent launch
constexpr int kSigInts = kSigQueue + 8 * 64;

// launch shape chosen for a GEMM (tile edge, K slices); exposed for the microbenchmark
struct GemmPlan { int tile, ksplit; };
GemmPlan gemm_plan(int epi, const GemmParams& p, int64_t ws_cap_doubles);
extern int g_gram_reg;   // 1: d in {1, 8, 16} Gram builds use the register-resident kernel; 2 (the
                         //    default): d in {8, 16} builds of every shape (square lower ones such
                         //    as K_ff and K̃mm included) on the matrix-core kernel — equal to 1
                         //    within the centred expansion's rounding, not bitwise (so K̃mm's
                         //    diagonal tiles are not bitwise symmetric there); d = 1 as in 1
extern int g_tiny_gemm;  // 1: the bottom-of-recursion GEMMs use the small kernel (gemm_plan)
extern int g_stream_k;   // stream-K tail of uniform-K 128-tile launches (launch_gemm): 0 never,
                         // 1 every eligible launch, 2 (default) those marked sk_alone
extern int g_slab_xcd;   // split-K launches: each XCD runs whole K slices (GPS_OPT_SLAB_XCD)
constexpr int kStreamKTiles = 4096;  // tickets per stream-K counter array (GemmParams::sk_cnt)

// ------------------------------------------------------------ device reductions
// fixed-order wave / block sums (no atomics anywhere: results are bitwise reproducible)
#ifdef __HIPCC__
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// block-wide sum of NV values per thread; result valid in every thread
template <int NV>
__device__ void block_sum(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = wave_sum(v[q]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) sh[q * 16 + wave] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += sh[q * 16 + w];
    v[q] = t;
  }
  __syncthreads();
}

// exp(x) for x <= 0 — the Gaussian kernel's exp(−½r²) — table-driven (round 4): x = (j/64)·ln2 + r
// with j = rint(64x/ln2), |r| <= ln2/128 (Cody–Waite: ln2/64 as a 35-bit head, exact for
// |j| <= 2^17, plus a tail), exp(x) = 2^(j>>6) · 2^((j&63)/64) · e^r, e^r − 1 by its degree-5
// Taylor polynomial (truncation 3.5e-17), 2^(i/64) as a head/tail pair (the table below, from
// 200-bit arithmetic).  About 12 fp64 VALU operations and one LDS read against ~25 for the
// library exp, whose overflow / underflow selects a non-positive argument never needs; within
// 1 ulp of exp.  x < −746 gives 0 (as exp), a NaN propagates.  The table is staged in LDS by
// each kernel (exp_tab_stage) so the per-lane index is a conflict-light ds_read_b128.
__constant__ static const double g_exp_tab[64][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0}, {0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56},
    {0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55}, {0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57},
    {0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54}, {0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59},
    {0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54}, {0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54},
    {0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55}, {0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55},
    {0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54}, {0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55},
    {0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54}, {0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55},
    {0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55}, {0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54},
    {0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55}, {0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54},
    {0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54}, {0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56},
    {0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55}, {0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58},
    {0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59}, {0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56},
    {0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56}, {0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54},
    {0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55}, {0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54},
    {0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54}, {0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54},
    {0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54}, {0x1.6623882552225p+0, -0x1.bb60987591c34p-54},
    {0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54}, {0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57},
    {0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55}, {0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54},
    {0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55}, {0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56},
    {0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54}, {0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54},
    {0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54}, {0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55},
    {0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57}, {0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54},
    {0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56}, {0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54},
    {0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54}, {0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54},
    {0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54}, {0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57},
    {0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56}, {0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55},
    {0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55}, {0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54},
    {0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56}, {0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54},
    {0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55}, {0x1.da9e603db3285p+0, 0x1.c2300696db532p-54},
    {0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54}, {0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55},
    {0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54}, {0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54},
    {0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54}, {0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55},
};
__device__ __forceinline__ void exp_tab_stage(double2* tab) {
  if (threadIdx.x < 64) tab[threadIdx.x] = make_double2(g_exp_tab[threadIdx.x][0], g_exp_tab[threadIdx.x][1]);
}
__device__ __forceinline__ double exp_neg(double x, const double2* tab) {
  x = x < -746.0 ? -746.0 : x;
  const double j = rint(x * 0x1.71547652b82fep+6);  // 64 / ln2
  const int n = (int)j;
  const double r = fma(-j, 0x1.1cf79abc9e3b4p-42, fma(-j, 0x1.62e42fef80000p-7, x));
  const double pr = r * fma(r, fma(r, fma(r, fma(r, 1.0 / 120.0, 1.0 / 24.0), 1.0 / 6.0), 0.5), 1.0);
  const double2 t = tab[n & 63];
  return ldexp(t.x + fma(t.x, pr, t.y), n >> 6);
}

// Gaussian CRPS and negative log density of one point (crps KF:60-68, logs KF:52-57; c is
// the VARIANCE)
__device__ __forceinline__ double crps_term(double m, double c, double y) {
  const double s = sqrt(c);
  const double z = (y - m) / s;
  const double cdf = 0.5 * (1.0 + erf(z * 0.70710678118654752440));
  const double pdf = 0.39894228040143267794 * exp(-z * z * 0.5);
  return s * (z * (2.0 * cdf - 1.0) + 2.0 * pdf - 0.56418958354775628695);
}
__device__ __forceinline__ double logs_term(double m, double c, double y) {
  const double e = y - m;
  return e * e / (2.0 * c) + log(sqrt(c)) + 0.91893853320467274178;
}
#endif

// gradient contraction: Σ_ij M_ij ∂A_ij/∂θ over the real n×n lower triangle with
// M_ij = a0·Ainv_ij + a1·α_iα_j + a2·½(v_iα_j + α_iv_j) + a3·Mx_ij (kernels_grad.hip)
struct GradParams {
  const double* x;          // [n][d] raw features
  int n, d;
  double sf2;
  double inv_ell[GPS_MAX_D];
  const double* Ainv; const double* Mx; int64_t ldm;
  const double* alpha; const double* v;
  double a0, a1, a2, a3;
  double* slab;             // grad_contract_slab_doubles(n, d)
};

// FITC gradient contraction (kernels_fitc_grad.hip): rows xr (nr), columns xc (nc),
// G_ij = Σ_t coef_t·(rs_t ? rs_t[i] : 1)·R_t[i][j] + Σ_q pc_q·pv_q[i]·qv_q[j]
struct FitcContractParams {
  const double* xr; const double* xc;   // [nr][d], [nc][d] raw features
  int nr, nc, nc_pad, d;
  double sf2;
  double inv_ell[GPS_MAX_D];
  int nt;                               // matrix terms (<= 4)
  const double* R[4]; int64_t ldr[4]; double coef[4]; const double* rs[4];
  double pc[2]; const double* pv[2]; const double* qv[2];  // rank-1 terms (pc = 0: off)
  double* slab;                         // fitc_contract_slab_doubles(nr, nc_pad, d)
  double* zslab;                        // set by the launcher
  int rchunk;                           // set by the launcher
};

// objective surfaces over a (length-scale, noise s.d.) grid (kernels_surface.hip, CP.R)
#define GPS_SURFACE_MAX_N 128
struct SurfaceParams {
  const double* x; const double* y;  // [n][d], [n]
  int n, d;
  double sf2;
  const double* ell; int nl;         // length-scales ℓ (not logs), grid columns
  const double* sd; int ns;          // noise standard deviations s (σ² = s²), grid rows
  int logs_add_noise;                // CP.R:81: LOO-LogS variance 1/d + s²
  double* out;                       // [4][ns][nl]: LOO-CRPS, in-sample CRPS, NLML, LOO-LogS
};

// ------------------------------------------------------------------ launchers
hipError_t launch_surface(const SurfaceParams& p, hipStream_t s);
hipError_t launch_gram(const GramParams& p, hipStream_t s);
// C = alpha * op(A) op(B) + beta * C with the epilogue selected by `epi`
hipError_t launch_gemm(int alay, int blay, int epi, const GemmParams& p, hipStream_t s);

// leaf of the recursive Cholesky: the diagonal 128×128 block, Cholesky + triangular inverse
// in one workgroup (kernels_potrf.hip).  Reads the lower triangle of A (lda), writes L⁻¹
// (lower, zeros above the diagonal) into Linv (ldl), L into Lout (optional), log(L_ii) into
// logdiag[0..127]; sets *info (atomicMin) to the 1-based global index of the first
// non-positive pivot.
hipError_t launch_potrf_leaf(const double* A, int64_t lda, double* Linv, int64_t ldl,
                             double* Lout, int64_t ldlo, double* logdiag, int* info,
                             int base, int n_real_in_block, hipStream_t s);

// persistent tiled factorisation of a diagonal block of T tiles (kernels_potrf.hip): L⁻¹ into
// Linv, L into A's strictly-lower tiles (and Lout if given), logdiag, info[0] as the leaf;
// info[1] != 0x7f7f7f7f on a lost dependency (bounded spin).  cnt: 16 + 2·T² ints, zero at the
// launch and left zero by it (its last workgroup resets them); tasks: dag_task_list(T, ..) on the device.
struct DagParams {
  double* A; int64_t lda;
  double* Linv; int64_t ldl;
  double* Lout; int64_t ldlo;
  double* logdiag; int* info; int base; int nreal;
  int T;
  const uint32_t* tasks; int ntasks;
  int* cnt;
  unsigned long long spin_ticks;   // 100 MHz s_memrealtime ticks a dependency wait may take
  unsigned long long* trace = nullptr;  // diagnostics only (tools/dag_bench.cpp): 4 words per slot
  int group = 3;                   // 16-deep operand chunks per load group of a strip task (2..4)
  int* sig = nullptr;              // row-ready signals for a dependent row-norm launch (kSig*):
                                   // +1 per started workgroup, row tile i flagged once L⁻¹'s row
                                   // tile i is final (LEAF(0); the last FIN(i, ·) strip)
};
hipError_t launch_potrf_dag(const DagParams& p, int nwg, hipStream_t s);
std::vector<uint32_t> dag_task_list(int T, int order = 1, bool fine = true);
inline int64_t dag_cnt_ints(int T) { return (16 + 2 * (int64_t)T * T + 63) / 64 * 64; }

// y[i] = sum_k L[i][k] x[k] over the tile-lower part (rows < n_pad)
hipError_t launch_gemv_lower(const double* L, int64_t ldl, const double* x, double* y,
                             int n_pad, hipStream_t s);
// y[i] = sum_k M[i][k] x[k], full rows
hipError_t launch_gemv_full(const double* M, int64_t ldm, const double* x, double* y,
                            int rows, int cols, hipStream_t s);
// column reductions over rows i (tile-lower if lower != 0):
//   s1[k] = sum_i M[i][k] w[i]   (if s1 != null)     s2[k] = sum_i M[i][k]^2 (if s2 != null)
// rowscale (optional) multiplies M[i][k] by rowscale[i] before both sums.
// Uses slab (>= nchunks*cols*2 doubles) and reduces into s1/s2.
hipError_t launch_colred(const double* M, int64_t ldm, int rows, int cols, int lower,
                         const double* w, const double* rowscale, double* s1, double* s2,
                         double* slab, hipStream_t s, int crows = 256);
// out[j] = sum_{s < nslab} slab[s*ld + j] (+ init[j] if init), j < len
hipError_t launch_slab_sum(const double* slab, int64_t ld, int nslab, int64_t len,
                           const double* init, double* out, hipStream_t s);
// sum of B slices into dst lower tiles + add (optional) base matrix; zero strict-upper tiles
hipError_t launch_sym_slab_sum(const double* slab, int64_t slice_stride, int nslab, int M,
                               const double* base, double* dst, hipStream_t s);

// symmetric m×m accumulator <-> lower-packed m(m+1)/2 (the FITC all-reduce payload):
// packed = Σ_q slab_q (lower, row-major; rows [r0, r1) only);  dst (M×M) = base +
// unpack(packed), lower 128-tiles (strict-upper tiles zero) or, with full, both triangles
hipError_t launch_sym_pack(const double* slab, int64_t slice_stride, int nslab, int r0, int r1,
                           int M, double* packed, hipStream_t s);
hipError_t launch_sym_unpack(const double* packed, int m, int M, const double* base, int full,
                             double* dst, hipStream_t s);
// full-GP LOO finalize (one workgroup): see kernels_vec.hip
// full-GP LOO: α, d = diag(A⁻¹) summed from the column pass's nslab chunk partials (slab:
// [α chunks | d chunks], ld apart), stored, then μ/σ² LOO and obj = [nlml, loo_crps, loo_logs,
// logdet, quad] (obj + 8: 4 scratch sums; part: ⌈n_pad/256⌉·4 doubles)
hipError_t launch_full_loo(const double* y, const double* slab, int nslab, int64_t ld,
                           const double* beta, const double* logdiag, int n, double* alpha,
                           double* dinv, double* mu_loo, double* var_loo, double* obj,
                           double* part, hipStream_t s);
// CP.R surface point from a resident fit: sums [Σ in-sample CRPS, Σ LOO-LogS (+ s² if add_noise)]
hipError_t launch_surface_point_sums(const double* y, const double* alpha, const double* dinv,
                                     int n, double s2, int add_noise, double* sums, double* part,
                                     hipStream_t s);
int launch_colred_partials(const double* M, int64_t ldm, int rows, int cols, int lower,
                           const double* w, double* slab, hipStream_t s);
// predictive variance finalize + test-score partial sums
hipError_t launch_pred_finalize(const double* s1, const double* s2, int nt, double base_var,
                                double* mu, double* var, hipStream_t s);
hipError_t launch_fitc_pred_finalize(const double* qm, const double* qb, int nt, double base_var,
                                     double* var, hipStream_t s);
// sums: [crps, logs, msll, sq_err, sq_err_trivial, cover]
// (part: scratch of ⌈nt/256⌉·6 doubles for the per-workgroup partials)
hipError_t launch_score_sums(const double* mu, const double* var, const double* y, int nt,
                             double ytr_mean, double ytr_var, double* sums, double* part,
                             hipStream_t s);
// FITC: q_i = Σ_t slab[t·ld + i] (nslab row-norm partials), λ_i = sf2 − q_i + σ² (real rows),
// 1 on pad rows; inv_lam = 1/λ; ys = y/λ; scalars: [Σ log λ, Σ y²/λ]
// (part: scratch of ⌈n_pad/256⌉·2 doubles)
hipError_t launch_fitc_lambda(const double* slab, int64_t ld, int nslab, const double* y, int n,
                              int n_pad, double sf2, double sn2, double* q, double* lam,
                              double* inv_lam, double* ys, double* scal, double* part,
                              hipStream_t s);
// FITC LOO: r_i = Σ_t slab[t·ld + i], d = 1/λ − r/λ², α = (y − g)/λ → μ, σ²; sums [Σ crps, Σ logs]
hipError_t launch_fitc_loo(const double* y, const double* lam, const double* slab, int64_t ld,
                           int nslab, const double* g, int n, int n_pad, double* r,
                           double* mu_loo, double* var_loo, double* sums, double* part,
                           hipStream_t s);
// small dense triangular mat-vec on the device: y = op(L) x with L lower (n_pad)
hipError_t launch_trmv_lower(const double* L, int64_t ldl, const double* x, double* y,
                             int n_pad, int trans, hipStream_t s);
hipError_t launch_dot(const double* a, const double* b, int n, double* out, hipStream_t s);
// dst (rows_pad × cols_pad) = src zero-padded; pad_identity puts 1 on the padded
// diagonal (embedding an SPD matrix as diag(A, I))
hipError_t launch_pad_copy(const double* src, int64_t lds, double* dst, int64_t ldd, int rows,
                           int cols, int rows_pad, int cols_pad, int pad_identity, hipStream_t s);

// --- gradients (kernels_grad.hip)
// u = −g_μ/d, ct = (g_μα − g_c)/d² of the mean LOO score `obj` (GPS_OBJ_LOO_CRPS / _LOGS)
hipError_t launch_loo_grad_terms(const double* y, const double* alpha, const double* dinv, int n,
                                 int n_pad, int obj, double* u, double* ct, hipStream_t s);
// strictly-upper 32-tiles := transpose of the strictly-lower ones
hipError_t launch_sym_mirror(double* M, int64_t ld, int n_pad, hipStream_t s);
// *out = max_i Σ_j |A_ij| over the n×n block (the ∞-norm; rowsum: n doubles of scratch)
hipError_t launch_norm_inf(const double* A, int64_t lda, int n, double* rowsum, double* out,
                           hipStream_t s);
int grad_contract_passes(int d);
int64_t grad_contract_slab_doubles(int n, int d);
// out[pass*18 + q]: q = 0 Σ w m K, 1 Σ_diag m, 2+k Σ w m K Δ²_(16·pass+k)
hipError_t launch_grad_contract(const GradParams& p, double* out, hipStream_t s);

// --- block-LOO (kernels_block.hip)
hipError_t launch_fold_terms(const double* y, const double* r, const double* c, int b, double* gm,
                             double* gc, double* out, hipStream_t s);
hipError_t launch_fold_grad(const double* PI, int64_t ldp, const double* H, int64_t ldh,
                            const double* r, const double* w, int b, double c0, double c1,
                            double c2, double c3, double gr, double gw, double* G, int64_t ldg,
                            double* g, hipStream_t s);
hipError_t launch_add_diag(double* P, int64_t ld, const double* vals, int nreal, int npad,
                           hipStream_t s);
hipError_t launch_row_scale(double* M, int64_t ld, int rows, int cols, const double* scale,
                            hipStream_t s);
hipError_t launch_vec_mul(const double* a, const double* b, int n, double* out, hipStream_t s);
// dst = base (+ base2) + sgn·Σ_{g ≠ skip} slab_g (len doubles, slabs `stride` apart, fixed order)
hipError_t launch_fold_sum(const double* slab, int64_t stride, int nslab, int skip, const double* base,
                           const double* base2, double sgn, double* dst, int64_t len, hipStream_t s);
// *out = Σ ldf[<m] − Σ ldb[<m] − ½Σ log lam[<b]: −½log|C_f| of a FITC block-LOO fold covariance
// the in-process communicator's device sum (kernels_vec.hip): up to kLocalSumMax ranks' staging
// buffers summed in rank order
constexpr int kLocalSumMax = 64;
struct LocalSumPtrs {
  const double* p[kLocalSumMax];
};
hipError_t launch_local_sum(const LocalSumPtrs& sp, int n, int64_t count, double* out, hipStream_t s);
// FITC block-LOO in low rank (kernels_block.hip): per-row dots of a b×m W, the fold vectors, and
// the F̃ rows as a base product plus rank-one terms
hipError_t launch_row_dots(const double* A, int64_t lda, const double* B, int64_t ldb,
                           const double* t, int rows, int cols, double* at, double* ab,
                           hipStream_t s);
hipError_t launch_lr_fold_vec(int mode, int b, int bp, const double* lam, const double* x,
                              const double* at, const double* ab, const double* r, const double* c,
                              const double* w, const double* gc, const double* q, double* o1,
                              double* o2, hipStream_t s);
hipError_t launch_lr_combine(const double* X, int64_t ldx, const double* Y, int64_t ldy,
                             const double* lam, const double* rs, double c0, const double* u1,
                             const double* v1, double c1, const double* u2, const double* v2,
                             double c2, int rows, int rows_pad, int cols, double* out, int64_t ldo,
                             hipStream_t s);
hipError_t launch_fold_logdet(const double* ldf, const double* ldb, int m, const double* lam, int b,
                              double* out, hipStream_t s);
// FITC block-LOO gradient (whitened): M_ii, the V Lm⁻¹ row scale and Y = −2Λ⁻¹F̃ + 2ŨS̃
// (see kernels_block.hip; Y may alias US)
hipError_t launch_blk_mdiag(const double* F, int64_t ldf, const double* US, int64_t ldus,
                            const double* U, int64_t ldu, int m_pad, const double* gd,
                            const double* lam, const double* v, const double* alpha, int n,
                            int n_pad, double* md, double* sc, double* Y, int64_t ldy,
                            hipStream_t s);
// energy score: Newton–Schulz steps, distances, reduction
hipError_t launch_ns_init(const double* C, int64_t ldc, int b, int bp, double scale, double pad,
                          double* Y, hipStream_t s);
hipError_t launch_diag_add_const(double* M, int64_t ld, int n, double c, hipStream_t s);
hipError_t launch_sym_avg(double* M, int64_t ld, int n, hipStream_t s);
hipError_t launch_scaled_row(const double* src, int b, int bp, double scale, double* dst,
                             hipStream_t s);
hipError_t launch_row_axpy(double* C, int64_t ldc, const double* Z, int64_t ldz, const double* sv,
                           int rows, int cols, hipStream_t s);
hipError_t launch_ns_resid(const double* T, int64_t ld, int n, double* out, hipStream_t s);
hipError_t launch_es_dist(const double* Z, const double* Zh, int64_t ld, int S, int bp, double* D,
                          int64_t ldd, hipStream_t s);
hipError_t launch_es_reduce(double* D, int64_t ldd, int S, int Sp, double beta, int grad,
                            double* rs, double* cs, double* out, hipStream_t s);

// --- FITC gradients (kernels_fitc_grad.hip)
hipError_t launch_fitc_grad_terms(const double* y, const double* lam, const double* r,
                                  const double* g, int n, int n_pad, int obj, double n_total,
                                  double* alpha, double* dinv, double* v, double* ulam, double* h,
                                  double* hl2, hipStream_t s);
hipError_t launch_fitc_grad_v(const double* ulam, const double* z, const double* lam, int n,
                              double* v, hipStream_t s);
hipError_t launch_fitc_grad_mdiag(const double* KN, int64_t ldkn, const double* K, int64_t ldk,
                                  int m_pad, const double* lam, const double* r, const double* dinv,
                                  const double* alpha, const double* v, const double* h, double a,
                                  int n, int n_pad, double* mdiag, double* s1, double* s2,
                                  double* s3, hipStream_t s);
hipError_t launch_fitc_grad_y(const double* U, const double* UP, int64_t ld, const double* s1,
                              const double* s2, int rows, int cols, double* Y, hipStream_t s);
int fitc_contract_passes(int d);
int64_t fitc_contract_slab_doubles(int nr, int nc_pad, int d);
// out[pass*17 + q]: q = 0 Σ GK, 1+k Σ GK Δ²_(16·pass+k);  zout[j*d + k] = Σ_i GK Δ_k (real j)
hipError_t launch_fitc_grad_contract(FitcContractParams p, double* out, double* zout,
                                     hipStream_t s);

}  // namespace gps
