// GEMM microbenchmark against libgpscore's internal launcher (gps::launch_gemm).
//   hipcc -O3 --offload-arch=gfx950 -I<pkg>/csrc tools/gemm_bench.cpp -L<pkg>/gpscore -lgpscore -o /tmp/gb
// Cases: square NT GEMM, the predictive TRMM shape, an L2-resident variant
// (lda = ldb = 0: every tile re-reads the same 16 KB, isolating the in-kernel
// pipeline from memory latency), and the recursion's small shapes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "gps_internal.h"
using namespace gps;

__global__ void fill_rand(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
    p[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

static double run(int al, int bl, int epi, GemmParams p, int reps, double flops) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  launch_gemm(al, bl, epi, p, 0);
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) launch_gemm(al, bl, epi, p, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return flops * reps / (ms * 1e-3) / 1e12;
}

// sweep: every recursion-level shape of the C3/C5 factorisation under each launch
// plan (tile 128/64 x split-K 1/2/4/8), to fit gemm_plan's thresholds
static int sweep(double* A, double* B, double* C, double* ws) {
  struct S { const char* name; int M, N, K, al, bl, tri, lower; } cs[] = {
    {"L5k tri1 NN", 5120, 4992, 5120, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L5k tri2 NT", 5120, 4992, 4992, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L5k tri3 NN", 5120, 4992, 4992, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"L5k syrk", 5120, 5120, 4992, LAY_N, LAY_T, TRI_NONE, 1},
    {"L2.5k tri1 NN", 2560, 2432, 2560, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L2.5k tri2 NT", 2560, 2432, 2432, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L2.5k tri3 NN", 2560, 2432, 2432, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"L2.5k syrk", 2560, 2560, 2432, LAY_N, LAY_T, TRI_NONE, 1},
    {"L2k tri1 NN", 2048, 2048, 2048, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L2k syrk", 2048, 2048, 2048, LAY_N, LAY_T, TRI_NONE, 1},
    {"L1280 tri1 NN", 1280, 1152, 1280, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L1280 tri2 NT", 1280, 1152, 1152, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L1280 tri3 NN", 1280, 1152, 1152, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"L1280 syrk", 1280, 1280, 1152, LAY_N, LAY_T, TRI_NONE, 1},
    {"L1k tri1 NN", 1024, 1024, 1024, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L1k syrk", 1024, 1024, 1024, LAY_N, LAY_T, TRI_NONE, 1},
    {"L640 tri1 NN", 640, 640, 640, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L640 tri2 NT", 640, 640, 640, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L640 syrk", 640, 640, 640, LAY_N, LAY_T, TRI_NONE, 1},
    {"L384 tri1 NN", 384, 256, 384, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L384 syrk", 384, 384, 256, LAY_N, LAY_T, TRI_NONE, 1},
    {"L256 tri1 NN", 256, 128, 256, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L256 syrk", 256, 256, 128, LAY_N, LAY_T, TRI_NONE, 1},
    {"L128 tri1 NN", 128, 128, 128, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L128 tri2 NT", 128, 128, 128, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L128 syrk", 128, 128, 128, LAY_N, LAY_T, TRI_NONE, 1},
  };
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs) {
    p.A = A; p.B = B; p.C = C; p.ws = ws;
    p.lda = c.al == LAY_N ? c.K : c.M;
    p.ldb = c.bl == LAY_T ? c.K : c.N;
    p.ldc = c.N;
    p.M = c.M; p.N = c.N; p.K = c.K; p.tri = c.tri; p.lower_out = c.lower;
    p.alpha = c.lower ? -1.0 : 1.0; p.beta = c.lower ? 1.0 : 0.0;
    const double fl = c.lower ? (double)c.M * (c.M + 1) * c.K : (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)c.K;
    const int reps = fl > 1e11 ? 10 : (fl > 1e9 ? 100 : 400);
    p.tile = 0; p.ksplit = 1;
    const GemmPlan auto_plan = gemm_plan(EPI_STORE, p, 1ll << 40);
    printf("%-16s auto(t%d,k%d) %7.2f |", c.name, auto_plan.tile, auto_plan.ksplit,
           run(c.al, c.bl, EPI_STORE, p, reps, fl));
    for (int tile : {128, 64})
      for (int ks : {1, 2, 4, 8}) {
        if (c.K / ks < 64) continue;
        p.tile = tile; p.ksplit = ks;
        const double t = run(c.al, c.bl, EPI_STORE, p, reps, fl);
        const double us = fl / (t * 1e12) * 1e6;
        printf(" t%d/k%d %6.2f (%6.1fus)", tile, ks, t, us);
      }
    printf("\n");
  }
  return 0;
}

// small-kernel study: the recursion's small shapes under the grouped-prefetch small kernel
// (block edge 16/32 × waves per block 1/2/4) against the 64-tile split-K plans; every variant
// is checked against the 128-tile single-slice result (max |diff|)
__global__ void maxdiff_kernel(const double* a, const double* b, int64_t n, int ncol, int lower, double* out) {
  double m = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (!lower || (i % ncol) / 64 <= (i / ncol) / 64) m = fmax(m, fabs(a[i] - b[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = m;
}
static double maxdiff(const double* a, const double* b, int64_t n, int ncol, int lower) {
  static double* d = nullptr;
  if (!d) hipMalloc(&d, 256 * 4 * 8);
  maxdiff_kernel<<<256, 256>>>(a, b, n, ncol, lower, d);
  double h[1024];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0.0;
  for (double v : h) m = fmax(m, v);
  return m;
}
static int small_study(double* A, double* B, double* C, double* ws) {
  struct S { const char* name; int M, N, K, al, bl, tri, lower; } cs[] = {
    {"L128 tri1 NN", 128, 128, 128, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L128 tri2 NT", 128, 128, 128, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L128 tri3 NN", 128, 128, 128, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"L128 syrk", 128, 128, 128, LAY_N, LAY_T, TRI_NONE, 1},
    {"L256 tri1 NN", 256, 128, 256, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L256 syrk", 256, 256, 128, LAY_N, LAY_T, TRI_NONE, 1},
    {"L256sq tri2 NT", 256, 256, 256, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L384 tri1 NN", 384, 256, 384, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L384 tri2 NT", 384, 256, 256, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L384 syrk", 384, 384, 256, LAY_N, LAY_T, TRI_NONE, 1},
    {"L512 tri2 NT", 512, 512, 512, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L512 syrk", 512, 512, 512, LAY_N, LAY_T, TRI_NONE, 1},
    {"L640 tri1 NN", 640, 640, 640, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L640 tri2 NT", 640, 640, 640, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"L640 tri3 NN", 640, 640, 640, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"L640 syrk", 640, 640, 640, LAY_N, LAY_T, TRI_NONE, 1},
    {"L1k tri1 NN", 1024, 1024, 1024, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L1k syrk", 1024, 1024, 1024, LAY_N, LAY_T, TRI_NONE, 1},
    {"L1280 tri1 NN", 1280, 1152, 1280, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"L1280 syrk", 1280, 1280, 1152, LAY_N, LAY_T, TRI_NONE, 1},
  };
  double* Cref;
  if (hipMalloc(&Cref, (int64_t)2048 * 2048 * 8) != hipSuccess) return 1;
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs) {
    p.A = A; p.B = B; p.ws = ws; p.ws_cap = 1ll << 28;
    p.lda = c.al == LAY_N ? c.K : c.M;
    p.ldb = c.bl == LAY_T ? c.K : c.N;
    p.ldc = c.N;
    p.M = c.M; p.N = c.N; p.K = c.K; p.tri = c.tri; p.lower_out = c.lower;
    p.alpha = -1.0; p.beta = 0.0;
    const double fl = c.lower ? (double)c.M * (c.M + 1) * c.K : (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)c.K;
    const int reps = 200;
    hipMemset(Cref, 0, (size_t)c.M * c.N * 8);
    p.C = Cref; p.tile = 128; p.ksplit = 1;
    launch_gemm(c.al, c.bl, EPI_STORE, p, 0);
    p.C = C;
    p.tile = 0; p.ksplit = 1;
    const GemmPlan ap = gemm_plan(EPI_STORE, p, p.ws_cap);
    double t = run(c.al, c.bl, EPI_STORE, p, reps, fl);
    printf("%-15s auto(t%d,k%d) %6.1fus |", c.name, ap.tile, ap.ksplit, fl / (t * 1e12) * 1e6);
    for (int tile : {64}) for (int ks : {1, 2, 4, 8}) {
      if (c.K / ks < 64) continue;
      p.tile = tile; p.ksplit = ks;
      t = run(c.al, c.bl, EPI_STORE, p, reps, fl);
      printf(" t64/k%d %6.1f", ks, fl / (t * 1e12) * 1e6);
    }
    printf(" |");
    for (int tile : {16, 32}) for (int w : {1, 2, 4}) {
      p.tile = tile; p.ksplit = w;
      hipMemset(C, 0, (size_t)c.M * c.N * 8);
      t = run(c.al, c.bl, EPI_STORE, p, reps, fl);
      const double d = maxdiff(C, Cref, (int64_t)c.M * c.N, c.N, c.lower);
      printf(" s%d/w%d %6.1f%s", tile, w, fl / (t * 1e12) * 1e6, d > 1e-9 ? "(BAD)" : "");
    }
    printf("\n");
  }
  return 0;
}

// leading-dimension study: the 10k-level shapes of the C3 build with the operands'
// real leading dimension (n_pad = 20096) against compact and padded alternatives
static int ldstudy(double* A, double* B, double* C) {
  struct S { const char* name; int M, N, K, al, bl, tri, lower; } cs[] = {
    {"K_LE_I NN 10112x9984x10112", 10112, 9984, 10112, LAY_N, LAY_N, TRI_K_LE_I, 0},
    {"K_LE_J NT 10112x9984x9984", 10112, 9984, 9984, LAY_N, LAY_T, TRI_K_LE_J, 0},
    {"K_GE_J NN 10112x9984x9984", 10112, 9984, 9984, LAY_N, LAY_N, TRI_K_GE_J, 0},
    {"SYRK NT 10112 K=9984", 10112, 10112, 9984, LAY_N, LAY_T, TRI_NONE, 1},
    {"TRMM-colred 20096x5120", 20096, 5120, 20096, LAY_N, LAY_T, TRI_K_LE_I, 0},
  };
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs) {
    for (int64_t ld : {0l, 20096l, 20160l, 20480l, 20608l}) {
      p.A = A; p.B = B; p.C = C;
      const int64_t lda0 = c.al == LAY_N ? c.K : c.M, ldb0 = c.bl == LAY_T ? c.K : c.N;
      p.lda = ld ? ld : lda0; p.ldb = ld ? ld : ldb0; p.ldc = ld ? ld : c.N;
      p.M = c.M; p.N = c.N; p.K = c.K; p.tri = c.tri; p.lower_out = c.lower;
      p.alpha = 1.0; p.beta = 0.0; p.ksplit = 1;
      const int64_t rowsA = c.al == LAY_N ? c.M : c.K, rowsB = c.bl == LAY_T ? c.N : c.K;
      if ((double)rowsA * p.lda > 20480.0 * 20480 || (double)rowsB * p.ldb > 20480.0 * 20480 ||
          (double)c.M * p.ldc > 20480.0 * 20480) { printf("%-28s ld %5ld skipped\n", c.name, (long)ld); continue; }
      const double fl = c.lower ? (double)c.M * (c.M + 1) * c.K : (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)c.K;
      printf("%-28s ld %5ld %7.2f TF/s\n", c.name, (long)(ld ? ld : lda0), run(c.al, c.bl, EPI_STORE, p, 3, fl));
    }
  }
  return 0;
}

// top-level trailing update of the C3 factorisation (3160 lower 128-tiles = 6.2 rounds of
// 512 resident workgroups): split-K through slabs vs the single launch
static int syrk_study(double* A, double* B, double* C) {
  double* ws;
  if (hipMalloc(&ws, (int64_t)4 * 10112 * 10112 * 8) != hipSuccess) return 1;
  GemmParams p; memset(&p, 0, sizeof(p));
  for (int M : {10112, 5120, 4992}) {
    const int K = M == 10112 ? 9984 : M;
    const double fl = (double)M * (M + 1) * K;
    for (int tile : {128, 64})
      for (int ks : {1, 2, 3, 4}) {
        p.A = A; p.B = A; p.C = C; p.lda = K; p.ldb = K; p.ldc = M;
        p.M = M; p.N = M; p.K = K; p.lower_out = 1; p.alpha = -1.0; p.beta = 1.0;
        p.tile = tile; p.ksplit = ks; p.ws = ks > 1 ? ws : nullptr; p.ws_cap = (int64_t)4 * 10112 * 10112;
        printf("SYRK M=%5d K=%5d t%3d ks%d %7.2f TF/s\n", M, K, tile, ks, run(LAY_N, LAY_T, EPI_STORE, p, 5, fl));
      }
  }
  return 0;
}

// layout study: the 10k-level triangular products of the C3 recursion in all four operand
// layouts (does storing T transposed / keeping L⁻ᵀ turn the NN products into faster ones?)
static int layout_study(double* A, double* B, double* C) {
  struct S { const char* name; int M, N, K, tri; } cs[] = {
    {"K_LE_I 10112x9984x10112", 10112, 9984, 10112, TRI_K_LE_I},
    {"K_GE_J 10112x9984x9984", 10112, 9984, 9984, TRI_K_GE_J},
    {"K_LE_J 10112x9984x9984", 10112, 9984, 9984, TRI_K_LE_J},
    {"K_LE_I 5120x4992x5120", 5120, 4992, 5120, TRI_K_LE_I},
    {"K_GE_J 5120x4992x4992", 5120, 4992, 4992, TRI_K_GE_J},
    {"NONE 8192^3", 8192, 8192, 8192, TRI_NONE},
  };
  const char* nm[2] = {"N", "T"};
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs)
    for (int al = 0; al < 2; ++al)
      for (int bl = 0; bl < 2; ++bl) {
        p.A = A; p.B = B; p.C = C; p.alpha = 1.0; p.beta = 0.0; p.ksplit = 1; p.tile = 0;
        p.lda = al == LAY_N ? c.K : c.M;
        p.ldb = bl == LAY_T ? c.K : c.N;
        p.ldc = c.N;
        p.M = c.M; p.N = c.N; p.K = c.K; p.tri = c.tri; p.lower_out = 0; p.map_mode = 0;
        const double fl = (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)c.K;
        printf("%-26s %s%s %7.2f TF/s\n", c.name, nm[al], nm[bl], run(al, bl, EPI_STORE, p, 5, fl));
      }
  return 0;
}

// FITC row-norm products ‖L⁻¹k_i‖² (EPI_ROWSQ, K ≤ j triangular) at the C4 / C5 shapes under
// every tile order: tall-skinny grids where each A row panel feeds all N/128 column tiles
static int rowsq_study(double* A, double* B, double* o0) {
  struct S { const char* name; int M, N; } cs[] = {
    {"C4 fit  40064x2048", 40064, 2048}, {"C4 pred 10112x2048", 10112, 2048},
    {"C5/2    100096x4096", 100096, 4096}};
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs)
    for (int mm : {0, 3, 1}) {  // auto (5), 3, grouped raster
      p.A = A; p.B = B; p.out0 = o0; p.alpha = 1.0; p.ksplit = 1; p.tile = 0;
      p.lda = c.N; p.ldb = c.N; p.ld_out = c.M;
      p.M = c.M; p.N = c.N; p.K = c.N; p.tri = TRI_K_LE_J; p.map_mode = mm;
      const double fl = (double)c.M * c.N * c.N;
      printf("rowsq %-22s map%d %7.2f TF/s\n", c.name, mm, run(LAY_N, LAY_T, EPI_ROWSQ, p, 5, fl));
    }
  return 0;
}

// where the row norms lose against the square products: the C4 fit shape as row norms and as a
// stored product, triangular K and full K, against the square 10k shape in both epilogues
static int rowsq_iso(double* A, double* B, double* C, double* o0) {
  struct S { const char* name; int M, N, epi, tri, mm, K = 0; } cs[] = {
    {"C4fit rowsq full K=1024", 40064, 2048, EPI_ROWSQ, TRI_NONE, 0, 1024},
    {"C4fit rowsq full K=512", 40064, 2048, EPI_ROWSQ, TRI_NONE, 0, 512},
    {"C4fit store full K=1024", 40064, 2048, EPI_STORE, TRI_NONE, 0, 1024},
    {"C4fit rowsq tri map5", 40064, 2048, EPI_ROWSQ, TRI_K_LE_J, 0},
    {"C4fit rowsq tri map3", 40064, 2048, EPI_ROWSQ, TRI_K_LE_J, 3},
    {"C4fit rowsq tri map6", 40064, 2048, EPI_ROWSQ, TRI_K_LE_J, 6},
    {"C4fit rowsqdot tri map6", 40064, 2048, EPI_ROWSQ_DOT, TRI_K_LE_J, 6},
    {"C4pred rowsq tri map5", 10112, 2048, EPI_ROWSQ, TRI_K_LE_J, 0},
    {"C4pred rowsq tri map6", 10112, 2048, EPI_ROWSQ, TRI_K_LE_J, 6},
    {"C5/2 rowsq tri map5", 100096, 4096, EPI_ROWSQ, TRI_K_LE_J, 0},
    {"C5/2 rowsq tri map6", 100096, 4096, EPI_ROWSQ, TRI_K_LE_J, 6},
    {"C4fit rowsq full", 40064, 2048, EPI_ROWSQ, TRI_NONE, 0},
    {"C4fit store tri map5", 40064, 2048, EPI_STORE, TRI_K_LE_J, 5},
    {"C4fit store tri map3", 40064, 2048, EPI_STORE, TRI_K_LE_J, 3},
    {"C4fit store full", 40064, 2048, EPI_STORE, TRI_NONE, 0},
    {"10k rowsq tri map5", 10112, 9984, EPI_ROWSQ, TRI_K_LE_J, 0},
    {"10k rowsq tri map3", 10112, 9984, EPI_ROWSQ, TRI_K_LE_J, 3},
    {"10k rowsq tri map6", 10112, 9984, EPI_ROWSQ, TRI_K_LE_J, 6},
    {"10k store tri map3", 10112, 9984, EPI_STORE, TRI_K_LE_J, 3},
    {"10k store tri map0", 10112, 9984, EPI_STORE, TRI_K_LE_J, 0},
  };
  GemmParams p;
  const int nc = sizeof(cs) / sizeof(cs[0]);
  for (int pass = 0; pass < 3; ++pass)  // forward, reversed, forward: clock ramp and drift show
  for (int ci = 0; ci < nc; ++ci)
    for (int prio = 0; prio < 1; ++prio) {  // (the wave-priority levels left the library in round 6)
      const S& c = cs[pass == 1 ? nc - 1 - ci : ci];
      memset(&p, 0, sizeof(p));
      p.A = A; p.B = B; p.C = C; p.out0 = o0; p.alpha = 1.0; p.ksplit = 1; p.tile = 0;
      const int K = c.K ? c.K : c.N;
      p.lda = K; p.ldb = K; p.ldc = c.N; p.ld_out = c.M;
      p.M = c.M; p.N = c.N; p.K = K; p.tri = c.tri; p.map_mode = c.mm;
      if (c.epi == EPI_ROWSQ_DOT) { p.w = o0 + 21 * (int64_t)c.M; p.out1 = o0 + 20 * (int64_t)c.M; }
      const double fl = (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)K;
      printf("p%d %-24s prio%d %7.2f TF/s\n", pass, c.name, prio, run(LAY_N, LAY_T, c.epi, p, 5, fl));
    }
  return 0;
}

// FITC split-K SYRK B = Kmnᵀ diag(λ⁻¹) Knm at the C4 / C5 shapes: the library's TN form (Knm
// row-major n×m, A transposed) against the NT form over a stored Kmn = Knmᵀ (m×n), with and
// without the per-k scale, and slice-major per XCD (g_slab_xcd)
static int fsyrk_study(double* A, double* C, double* w) {
  double* ws;
  if (hipMalloc(&ws, (int64_t)24 * 4096 * 4096 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(fill_rand, dim3(64), dim3(256), 0, 0, w, (int64_t)200064, 3ull);
  // (operands: A holds n*n = 419M doubles; 4096 x 100032 = 410M fit)
  struct S { const char* name; int m, n, ks; } cs[] = {{"C4 2048 K=40064", 2048, 40064, 11},
                                                       {"C5/2 4096 K=100032", 4096, 100032, 13}};
  GemmParams p; memset(&p, 0, sizeof(p));
  for (auto& c : cs)
    for (int lay = 0; lay < 2; ++lay)
      for (int ksc = 0; ksc < 2; ++ksc)
        for (int sx = 0; sx < 2; ++sx) {
          memset(&p, 0, sizeof(p));
          p.A = A; p.B = A; p.C = C; p.ws = ws; p.ws_cap = (int64_t)24 * 4096 * 4096;
          p.M = c.m; p.N = c.m; p.K = c.n; p.lower_out = 1; p.ksplit = c.ks; p.alpha = 1.0; p.ldc = c.m;
          p.kscale = ksc ? w : nullptr;
          const int al = lay == 0 ? LAY_T : LAY_N, bl = lay == 0 ? LAY_N : LAY_T;
          p.lda = lay == 0 ? c.m : c.n; p.ldb = p.lda;
          g_slab_xcd = sx;
          const double fl = (double)c.m * (c.m + 1) * c.n;
          printf("fsyrk %-18s %s kscale%d sxcd%d %7.2f TF/s\n", c.name, lay == 0 ? "TN" : "NT", ksc, sx,
                 run(al, bl, EPI_STORE, p, 5, fl));
        }
  g_slab_xcd = 0;
  return 0;
}

int main(int argc, char** argv) {
  const int64_t n = 20480;
  double *A, *B, *C, *o0, *o1, *w;
  hipMalloc(&A, n * n * 8); hipMalloc(&B, n * n * 8); hipMalloc(&C, n * n * 8);
  hipMalloc(&o0, 64 * 200064 * 8); hipMalloc(&o1, 256 * n * 8); hipMalloc(&w, 200064 * 8);
  const bool zeros = getenv("GB_ZEROS") != nullptr;
  if (zeros) { hipMemset(A, 0, n * n * 8); hipMemset(B, 0, n * n * 8); }
  else {
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, n * n, 1ull);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, n * n, 2ull);
  }
  hipMemset(w, 0, n * 8);
  printf("operands: %s\n", zeros ? "zeros" : "uniform random [-0.5, 0.5)");
  if (argc > 1 && !strcmp(argv[1], "ld")) return ldstudy(A, B, C);
  if (argc > 1 && !strcmp(argv[1], "small")) {
    double* ws; hipMalloc(&ws, (int64_t)8 << 28);
    return small_study(A, B, C, ws);
  }
  if (argc > 1 && !strcmp(argv[1], "syrk")) return syrk_study(A, B, C);
  if (argc > 1 && !strcmp(argv[1], "layout")) return layout_study(A, B, C);
  if (argc > 1 && !strcmp(argv[1], "rowsq")) return rowsq_study(A, B, o0);
  if (argc > 1 && !strcmp(argv[1], "rowsq_iso")) return rowsq_iso(A, B, C, o0);
  if (argc > 1 && !strcmp(argv[1], "fsyrk")) return fsyrk_study(A, C, w);
  if (argc > 1 && !strcmp(argv[1], "sweep")) {
    double* ws; hipMalloc(&ws, (int64_t)8 * 5120 * 5120 * 8);
    return sweep(A, B, C, ws);
  }
  GemmParams p; memset(&p, 0, sizeof(p)); p.alpha = 1; p.ksplit = 1;
  struct { const char* name; int M, N, K, al, bl, epi, tri, lower, l2; } cs[] = {
    {"NT 8192^3", 8192, 8192, 8192, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 8192^3 L2-resident", 8192, 8192, 8192, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 1},
    {"NN 8192^3", 8192, 8192, 8192, LAY_N, LAY_N, EPI_STORE, TRI_NONE, 0, 0},
    {"TN 4096x4096 K=40960", 4096, 4096, 40960 / 2, LAY_T, LAY_N, EPI_STORE, TRI_NONE, 0, 0},
    {"SYRK NT 10112 K=9984", 10112, 10112, 9984, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 1, 0},
    {"TRMM-colred 20096x5120", 20096, 5120, 20096, LAY_N, LAY_T, EPI_COLRED, TRI_K_LE_I, 0, 0},
    {"TRMM-colred L2-resident", 20096, 5120, 20096, LAY_N, LAY_T, EPI_COLRED, TRI_K_LE_I, 0, 1},
    {"NT 20096x5120x20096 store", 20096, 5120, 20096, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 20096x5120 tri store", 20096, 5120, 20096, LAY_N, LAY_T, EPI_STORE, TRI_K_LE_I, 0, 0},
    {"NT 20096x5120 colred notri", 20096, 5120, 20096, LAY_N, LAY_T, EPI_COLRED, TRI_NONE, 0, 0},
    {"NT 5120x20096x20096 store", 5120, 20096, 20096, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"K_LE_J NT 10112x9984x9984", 10112, 9984, 9984, LAY_N, LAY_T, EPI_STORE, TRI_K_LE_J, 0, 0},
    {"K_GE_J NN 10112x9984x9984", 10112, 9984, 9984, LAY_N, LAY_N, EPI_STORE, TRI_K_GE_J, 0, 0},
    {"K_LE_I NN 10112x9984x10112", 10112, 9984, 10112, LAY_N, LAY_N, EPI_STORE, TRI_K_LE_I, 0, 0},
    {"SYRK NT 5120 K=5120", 5120, 5120, 5120, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 1, 0},
    {"NT 5120^3", 5120, 5120, 5120, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 2560^3", 2560, 2560, 2560, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 1280^3", 1280, 1280, 1280, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 640x640x640", 640, 640, 640, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
    {"NT 256^3", 256, 256, 256, LAY_N, LAY_T, EPI_STORE, TRI_NONE, 0, 0},
  };
  for (auto& c : cs) {
    p.A = A; p.B = B; p.C = C; p.w = w; p.out0 = o0; p.out1 = o1;
    p.lda = c.l2 ? 0 : (c.al == LAY_N ? c.K : c.M);
    p.ldb = c.l2 ? 0 : (c.bl == LAY_T ? c.K : c.N);
    p.ldc = c.N; p.ld_out = c.epi == EPI_ROWSQ ? c.M : c.N;
    p.M = c.M; p.N = c.N; p.K = c.K; p.tri = c.tri; p.lower_out = c.lower;
    // every operand must lie inside its n*n allocation (an out-of-bounds read can fault the GPU)
    if ((double)c.M * c.K > (double)n * n || (double)c.K * c.N > (double)n * n ||
        (double)c.M * c.N > (double)n * n) { printf("%-28s skipped (too big)\n", c.name); continue; }
    double fl = c.lower ? (double)c.M * (c.M + 1) * c.K : (c.tri ? 1.0 : 2.0) * c.M * c.N * (double)c.K;
    int reps = fl > 1e12 ? 3 : (fl > 1e10 ? 20 : 200);
    for (int mm = 0; mm < 4; ++mm) {
      if (!c.tri && !c.lower && mm) continue;
      if (mm == 3 && !c.tri) continue;
      p.map_mode = mm;
      printf("%-28s map%d %7.2f TF/s\n", c.name, mm, run(c.al, c.bl, c.epi, p, reps, fl));
    }
    if (c.lower) {
      p.map_mode = 0; p.tile = 64;
      printf("%-28s t64  %7.2f TF/s\n", c.name, run(c.al, c.bl, c.epi, p, reps, fl));
      p.tile = 0;
    }
  }
  return 0;
}
