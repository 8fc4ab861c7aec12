// Gram-build microbenchmark (round 5): the library's d = 8 Gram (csrc/kernels_gram.hip: the
// direct-difference gram_reg_kernel<8> until the matrix-core gram_mfma_kernel<8, true> replaced it)
// on the C3 shapes — K_ff lower (20000², d = 8) and K*f (5000 × 20000) — against variants of the
// register kernel's interior-tile loop on the K*f shape (store-only: the access pattern's ceiling,
// 256 columns per workgroup, 64 rows per workgroup, 4 rows per unrolled step; bitwise check
// against the library, which only holds while the library is that kernel) and store-only kernels
// with the matrix-core kernel's output layout (profiles/r5ap_gram_bench.txt: 5.39 TB/s, the
// 16-byte-row pattern 5.50).
//   hipcc -O3 --offload-arch=gfx950 -I include -I <pkg>/csrc tools/gram_bench.cpp -o tbin/gram_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "kernels_gram.hip"
using namespace gps;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// interior-tile variant: ROWS × COLS tile, COLS / 128 column pairs per lane, UNR rows per step
template <int D, int COLS, int ROWS, int UNR, bool STORE_ONLY>
__global__ __launch_bounds__(256) void gram_var(GramParams p) {
  constexpr int CP = COLS / 128;  // column pairs per lane
  __shared__ __attribute__((aligned(16))) double xs_row[ROWS * D];
  __shared__ double2 etab[64];
  const int tiles_x = p.N / COLS;
  const int c0 = (blockIdx.x % tiles_x) * COLS, r0 = (blockIdx.x / tiles_x) * ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < ROWS * D; e += 256) {
    const int i = e / D, k = e - i * D;
    xs_row[e] = p.x[(int64_t)(r0 + i) * D + k] * p.inv_ell[k];
  }
  double f[CP][2][D];
#pragma unroll
  for (int c = 0; c < CP; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < D; ++k) f[c][h][k] = p.xp[(int64_t)(c0 + 128 * c + 2 * lane + h) * D + k] * p.inv_ell[k];
  exp_tab_stage(etab);
  __syncthreads();
#pragma unroll UNR
  for (int rr = wave; rr < ROWS; rr += 4) {
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      double a0 = 0.0, a1 = 0.0;
      if constexpr (!STORE_ONLY) {
#pragma unroll
        for (int k = 0; k < D; k += 2) {
          const double2 xr = *reinterpret_cast<const double2*>(&xs_row[rr * D + k]);
          double e0 = xr.x - f[c][0][k], e1 = xr.x - f[c][1][k];
          a0 = fma(e0, e0, a0);
          a1 = fma(e1, e1, a1);
          e0 = xr.y - f[c][0][k + 1];
          e1 = xr.y - f[c][1][k + 1];
          a0 = fma(e0, e0, a0);
          a1 = fma(e1, e1, a1);
        }
      }
      double* dst = p.out + (int64_t)(r0 + rr) * p.ldo + c0 + 128 * c + 2 * lane;
      if constexpr (STORE_ONLY)
        st_nt2(dst, p.sf2, p.sf2);
      else
        st_nt2(dst, p.sf2 * exp_neg(-0.5 * a0, etab), p.sf2 * exp_neg(-0.5 * a1, etab));
    }
  }
}


// One column per lane (the library keeps two: at d = 16 that is 64 VGPRs of features, 122 in all,
// 4 waves per SIMD); the expansion form ‖x‖² + ‖z‖² − 2x·z drops the per-feature subtraction
// (reported as max |diff| against the library: it is not the library's arithmetic).  ROWS rows
// per workgroup, UNR rows per unrolled step.
template <int D, bool EXPAND, int UNR, int ROWS>
__global__ __launch_bounds__(256) void gram_one_col(GramParams p) {
  __shared__ __attribute__((aligned(16))) double xs_row[ROWS * D];
  __shared__ double rn[ROWS];
  __shared__ double2 etab[64];
  const int tiles_x = p.N / GR_COLS;
  const int c0 = (blockIdx.x % tiles_x) * GR_COLS, r0 = (blockIdx.x / tiles_x) * ROWS;
  const int tid = threadIdx.x;
  for (int e = tid; e < ROWS * D; e += 256) {
    const int i = e / D, k = e - i * D;
    xs_row[e] = p.x[(int64_t)(r0 + i) * D + k] * p.inv_ell[k];
  }
  const int gj = c0 + (tid & 127), half = tid >> 7;
  double f[D], fn = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    f[k] = p.xp[(int64_t)gj * D + k] * p.inv_ell[k];
    fn = fma(f[k], f[k], fn);
  }
  exp_tab_stage(etab);
  __syncthreads();
  if (EXPAND) {
    for (int r = tid; r < ROWS; r += 256) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) s = fma(xs_row[r * D + k], xs_row[r * D + k], s);
      rn[r] = s;
    }
    __syncthreads();
  }
  // waves 0 / 1 hold columns 0-63 / 64-127 for the even rows, waves 2 / 3 for the odd rows
#pragma unroll UNR
  for (int rr = half; rr < ROWS; rr += 2) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < D; k += 2) {
      const double2 xr = *reinterpret_cast<const double2*>(&xs_row[rr * D + k]);
      if (EXPAND) {
        a = fma(xr.x, f[k], a);
        a = fma(xr.y, f[k + 1], a);
      } else {
        double e = xr.x - f[k];
        a = fma(e, e, a);
        e = xr.y - f[k + 1];
        a = fma(e, e, a);
      }
    }
    if (EXPAND) a = fmax(fma(-2.0, a, rn[rr] + fn), 0.0);
    __builtin_nontemporal_store(p.sf2 * exp_neg(-0.5 * a, etab), p.out + (int64_t)(r0 + rr) * p.ldo + gj);
  }
}

// store-only with the matrix-core kernel's output layout: per 16-column block each lane stores
// 8 bytes to 4 rows (v_mfma_f64_16x16x4 accumulator order: 4 × 128 contiguous bytes per store
// instruction); PAIR: lane pairs swap halves first (one __shfl_xor) so that each lane stores 16
// bytes to 2 rows (2 × 256 bytes per instruction)
template <bool PAIR>
__global__ __launch_bounds__(256) void store_mfma_layout(GramParams p) {
  const int tiles_x = p.N / 128;
  const int c0 = (blockIdx.x % tiles_x) * 128, r0 = (blockIdx.x / tiles_x) * 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15, lg = lane >> 4;
  double* const obase = p.out + (int64_t)(r0 + 32 * wave) * p.ldo + c0;
  for (int cb = 0; cb < 8; ++cb)
    for (int rb = 0; rb < 2; ++rb) {
      double v[4];
      for (int q = 0; q < 4; ++q) v[q] = p.sf2 + q + lr;
      if constexpr (PAIR) {
        // even lane keeps rows q = 0,1 and takes the odd lane's, odd lane rows 2,3
        const bool odd = lr & 1;
        const double s0 = __shfl_xor(odd ? v[0] : v[2], 1), s1 = __shfl_xor(odd ? v[1] : v[3], 1);
        const int c = 16 * cb + (lr & ~1);
        typedef double nv2 __attribute__((ext_vector_type(2)));
        for (int h = 0; h < 2; ++h) {
          const int q = odd ? 2 + h : h;
          const double mine = v[q], other = h ? s1 : s0;
          const nv2 pr = odd ? (nv2){other, mine} : (nv2){mine, other};
          __builtin_nontemporal_store(pr, reinterpret_cast<nv2*>(obase + (int64_t)(16 * rb + 4 * q + lg) * p.ldo + c));
        }
      } else {
        for (int q = 0; q < 4; ++q)
          __builtin_nontemporal_store(v[q], obase + (int64_t)(16 * rb + 4 * q + lg) * p.ldo + 16 * cb + lr);
      }
    }
}

__global__ void maxdiff_k(const double* a, const double* b, int64_t n, double* out) {
  double m = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmax(m, fabs(a[i] - b[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = m;
}

// plain (interior) Gram of n × m at feature count D: the library against the one-column variants
template <int D>
static void col_study(int n, int m) {
  std::mt19937_64 rng(5);
  std::normal_distribution<double> nd;
  std::vector<double> hx((size_t)n * D), hz((size_t)m * D);
  for (auto& v : hx) v = nd(rng);
  for (auto& v : hz) v = nd(rng);
  double *X, *Zp, *ref, *out, *md;
  CK(hipMalloc(&X, hx.size() * 8)); CK(hipMalloc(&Zp, hz.size() * 8));
  CK(hipMalloc(&ref, (size_t)n * m * 8)); CK(hipMalloc(&out, (size_t)n * m * 8)); CK(hipMalloc(&md, 1024 * 8));
  CK(hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Zp, hz.data(), hz.size() * 8, hipMemcpyHostToDevice));
  GramParams g;
  memset(&g, 0, sizeof(g));
  g.d = D; g.sf2 = 1.3; g.x = X; g.xp = Zp; g.ldo = m; g.n = n; g.m = m; g.M = n; g.N = m;
  for (int k = 0; k < D; ++k) g.inv_ell[k] = 1.0 / (2.0 + 0.1 * k);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 8.0 * n * m;
  auto time = [&](auto launch, const char* name) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("d%-2d %6d x %5d %-34s %8.4f ms  %6.0f GB/s\n", D, n, m, name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  GramParams r = g; r.out = ref;
  time([&] { CK(launch_gram(r, 0)); }, "library");
  GramParams v = g; v.out = out;
  auto check = [&](const char* name) {
    hipLaunchKernelGGL(maxdiff_k, dim3(256), dim3(256), 0, 0, out, ref, (int64_t)n * m, md);
    std::vector<double> h(1024);
    CK(hipMemcpy(h.data(), md, 1024 * 8, hipMemcpyDeviceToHost));
    double mx = 0.0;
    for (double x : h) mx = fmax(mx, x);
    printf("    %s: max |diff| vs library %.3e\n", name, mx);
    CK(hipMemset(out, 0, (size_t)n * m * 8));
  };
#define OC(EX, UNR, ROWS, NAME)                                                                    \
  time([&] { hipLaunchKernelGGL((gram_one_col<D, EX, UNR, ROWS>), dim3((n / ROWS) * (m / GR_COLS)), \
                                dim3(256), 0, 0, v); }, NAME);                                     \
  check(NAME);
  OC(false, 1, 128, "one col, unroll 1, 128 rows")
  OC(false, 2, 128, "one col, unroll 2, 128 rows")
  OC(false, 4, 128, "one col, unroll 4, 128 rows")
  OC(false, 2, 256, "one col, unroll 2, 256 rows")
  OC(false, 2, 64, "one col, unroll 2, 64 rows")
  OC(true, 2, 128, "one col, expansion, unroll 2")
#undef OC
  CK(hipFree(X)); CK(hipFree(Zp)); CK(hipFree(ref)); CK(hipFree(out)); CK(hipFree(md));
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  if (argc > 1 && !strcmp(argv[1], "cols")) {
    col_study<16>(100096, 4096);
    col_study<8>(5120, 20096);
    return 0;
  }
  const int d = 8, n = 20096, nt = 5120;  // padded C3 sizes (all tiles interior for K*f)
  std::mt19937_64 rng(3);
  std::normal_distribution<double> nd;
  std::vector<double> hx((size_t)n * d), ht((size_t)nt * d);
  for (auto& v : hx) v = nd(rng);
  for (auto& v : ht) v = nd(rng);
  double *X, *Xt, *out, *ref;
  CK(hipMalloc(&X, hx.size() * 8)); CK(hipMalloc(&Xt, ht.size() * 8));
  CK(hipMalloc(&out, (size_t)n * n * 8)); CK(hipMalloc(&ref, (size_t)nt * n * 8));
  CK(hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xt, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
  GramParams g;
  memset(&g, 0, sizeof(g));
  g.d = d; g.sf2 = 1.0;
  for (int k = 0; k < d; ++k) g.inv_ell[k] = 0.5;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](auto launch, double bytes, const char* name) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-34s %8.4f ms  %6.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  // library: K_ff lower (n × n) and K*f (nt × n)
  GramParams kff = g;
  kff.x = X; kff.xp = X; kff.out = out; kff.ldo = n; kff.n = n; kff.m = n; kff.M = n; kff.N = n;
  kff.lower = 1; kff.diag_add = 0.01; kff.pad_identity = 1;
  time([&] { CK(launch_gram(kff, 0)); }, 8.0 * n * (n + 1.0) / 2, "library K_ff lower 20096^2");
  GramParams ksf = g;
  ksf.x = Xt; ksf.xp = X; ksf.out = ref; ksf.ldo = n; ksf.n = nt; ksf.m = n; ksf.M = nt; ksf.N = n;
  time([&] { CK(launch_gram(ksf, 0)); }, 8.0 * nt * n, "library K*f 5120 x 20096");
  const double bsf = 8.0 * nt * n;
  GramParams v = ksf;
  v.out = out;
  auto check = [&](const char* name) {
    std::vector<double> a((size_t)nt * n), b((size_t)nt * n);
    CK(hipMemcpy(a.data(), out, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), ref, b.size() * 8, hipMemcpyDeviceToHost));
    printf("    %s: %s\n", name, memcmp(a.data(), b.data(), a.size() * 8) ? "DIFFERS" : "bitwise equal");
  };
#define VAR(COLS, ROWS, UNR, SO, NAME)                                                           \
  time([&] { hipLaunchKernelGGL((gram_var<8, COLS, ROWS, UNR, SO>),                             \
                                dim3((nt / ROWS) * (n / COLS)), dim3(256), 0, 0, v); }, bsf, NAME); \
  if (!SO) check(NAME);
  VAR(128, 128, 2, true, "store-only 128x128");
  time([&] { hipLaunchKernelGGL(store_mfma_layout<false>, dim3((nt / 128) * (n / 128)), dim3(256), 0, 0, v); },
       bsf, "store-only mfma layout (4 x 128 B)");
  time([&] { hipLaunchKernelGGL(store_mfma_layout<true>, dim3((nt / 128) * (n / 128)), dim3(256), 0, 0, v); },
       bsf, "store-only mfma layout, pairs (2 x 256 B)");
  VAR(128, 128, 2, false, "variant 128x128 unroll 2 (=lib)");
  VAR(128, 128, 4, false, "variant 128x128 unroll 4");
  VAR(128, 64, 2, false, "variant 64 rows x 128");
  VAR(128, 256, 2, false, "variant 256 rows x 128");
  if (n % 256 == 0) { VAR(256, 128, 2, false, "variant 128 x 256 cols"); }
  return 0;
}
