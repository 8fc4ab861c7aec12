// Where the 128-block leaf's time goes, phase by phase and wave by wave: a timing-only copy of
// v4::leaf_body (csrc/kernels_potrf.hip) with s_memtime stamps (shader clock) taken by lane 0 of
// every wave at each phase boundary, plus SKIP variants that drop one kind of work (results are
// then wrong; only the stamps matter).  One workgroup, the stand-alone (non-coherent) form.
//   leaf_probe [reps=50] [which=0: SKIP variants, 1: batched phase-A tiles]
// SKIP bits: 1 the pivot panel, 2 phase A's trailing tile updates, 4 the inverse (diag inverse,
// T_k products, X finish, tail), 8 phase B's look-ahead column update.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "kernels_potrf.hip"
using namespace gps;
using namespace gps::v4;

constexpr int NST = 40;  // stamps per wave

// (the batched phase-A deal: v4::g_deal / tile_update_group in kernels_potrf.hip)
template <int SKIP, int BATCH, bool UNI>
__global__ __launch_bounds__(256) void leaf_probe_kernel(const double* __restrict__ A, int64_t lda,
                                                          double* __restrict__ Linv, int64_t ldl,
                                                          double* __restrict__ logdiag,
                                                          unsigned long long* stamps) {
  __shared__ double S[NT * TSZ];
  __shared__ double DG[128];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = UNI ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  unsigned long long* my = stamps + wave * NST;
  auto stamp = [&](int i) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (lane == 0) my[i] = t;
  };
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  stamp(0);
  {
    const int hb = tid >> 7, q = tid & 127, r = q >> 3, c2 = (q & 7) * 2;
    dv2 v[18];
#pragma unroll
    for (int m = 0; m < 18; ++m) {
      const int ti = hb ? tile_i(2 * m + 1) : tile_i(2 * m);
      const int tj = hb ? 2 * m + 1 - tix(tile_i(2 * m + 1), 0) : 2 * m - tix(tile_i(2 * m), 0);
      v[m] = ld_d2<false>(A + (int64_t)(16 * ti + r) * lda + 16 * tj + c2);
    }
#pragma unroll
    for (int m = 0; m < 18; ++m) {
      const int t = 2 * m + hb;
      S[t * TSZ + r * TS + c2] = v[m].x;
      S[t * TSZ + r * TS + c2 + 1] = v[m].y;
    }
  }
  __syncthreads();
  stamp(1);
  d4 T[3];
  const int uw = wave - 1;
  for (int p = 0; p < 8; ++p) {
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
      if (!(SKIP & 1)) {
        if (p < 4) factor_panel<0, true>(P, p, lane);
        else factor_panel<1, false>(P, p, lane);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R = lane + 64 * s;
        if (R >= t0) {
          const int t = tix(R >> 4, p) * TSZ + (R & 15) * TS;
#pragma unroll
          for (int c = 0; c < 16; ++c) S[t + c] = P[s][c];
        }
      }
    } else if (p >= 1) {
      const int pp = p - 1;
      const int winv = pp % 3;
      const int rank = (uw - winv + 3) % 3;
      int task = 0;
      if constexpr (BATCH > 0) {
        if (!(SKIP & 2)) {
          const int n = g_deal.n[p][rank];
          for (int g0 = 0; g0 < n; g0 += BATCH)
            tile_update_group<BATCH>(S, g_deal.t[p][rank] + g0, n - g0, lane);
        }
      } else if (!(SKIP & 2)) {
        for (int j = p + 1; j < 8; ++j)
          for (int i = j; i < 8; ++i, ++task) {
            const int who = task % 5 == 4 ? 0 : 1 + ((task - task / 5) & 1);
            if (who == rank) tile_update(S, tix(i, j), tix(i, pp), tix(j, pp), lane);
          }
      }
      if (!(SKIP & 4)) {
        if (rank == 0) {
          invert_diag<false>(S, DG, pp, lane, Linv, ldl);
          if (lane < 16) logdiag[16 * pp + lane] = log(DG[16 * pp + lane]);
        }
#pragma unroll
        for (int slot = 0; slot < 3; ++slot) {
          const int k = uw + 3 * slot;
          if (k < pp) T[slot] = inv_row_t(S, pp, k, lane);
        }
      }
    }
    stamp(2 + 4 * p);
    __syncthreads();
    stamp(3 + 4 * p);
    if (p < 7) {
      if (!(SKIP & 8)) {
        const int i0 = p + 1 + wave, i1 = p + 5 + wave, tb = tix(p + 1, p);
        if (i1 < 8) tile_update2(S, tix(i0, p + 1), tix(i0, p), tix(i1, p + 1), tix(i1, p), tb, lane);
        else if (i0 < 8) tile_update(S, tix(i0, p + 1), tix(i0, p), tb, lane);
      }
    } else if (wave == 0 && !(SKIP & 4)) {
      invert_diag<false>(S, DG, 7, lane, Linv, ldl);
    }
    if (p >= 1 && wave != 0 && !(SKIP & 4)) {
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
    stamp(4 + 4 * p);
    __syncthreads();
    stamp(5 + 4 * p);
  }
  if (!(SKIP & 4)) {
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int k = tail_k(wave, slot);
      if (k >= 0) T[slot] = inv_row_t(S, 7, k, lane);
    }
  }
  stamp(34);
  __syncthreads();
  stamp(35);
  if (!(SKIP & 4)) {
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
  stamp(36);
  {
    const int hb = tid >> 7, q = tid & 127, r = q >> 3, c2 = (q & 7) * 2;
#pragma unroll
    for (int m = 0; m < 14; ++m) {
      const int u = 2 * m + hb;
      const int ui = u < 7 ? 0 : u < 13 ? 1 : u < 18 ? 2 : u < 22 ? 3 : u < 25 ? 4 : u < 27 ? 5 : 6;
      const int ustart = ui * 7 - ui * (ui - 1) / 2;
      const int uj = ui + 1 + (u - ustart);
      st_d2<false>(Linv + (int64_t)(16 * ui + r) * ldl + 16 * uj + c2, (dv2){0.0, 0.0});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(37);
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) { my[38] = 0; my[39] = rt1 - rt0; }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int SKIP, int BATCH = 0, bool UNI = false>
static void probe(const double* A, double* Li, double* ld, unsigned long long* st, int reps) {
  const int n = 128;
  std::vector<double> acc(4 * NST, 0.0);
  std::vector<unsigned long long> h(4 * NST);
  for (int r = 0; r < reps + 5; ++r) {
    leaf_probe_kernel<SKIP, BATCH, UNI><<<dim3(1), dim3(256), 0, 0>>>(A, n, Li, n, ld, st);
    CK(hipDeviceSynchronize());
    if (r < 5) continue;
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    const unsigned long long t0 = h[0];
    for (int i = 0; i < 4 * NST; ++i) acc[i] += i % NST >= 38 ? (double)h[i] : (double)(h[i] - t0);
  }
  for (auto& a : acc) a /= reps;
  auto at = [&](int w, int i) { return acc[w * NST + i]; };
  printf("SKIP=%d BATCH=%d UNI=%d: total %.0f cycles = %.2f us (100 MHz clock: %.0f cycles/us); load+sync %.0f\n", SKIP, BATCH, (int)UNI,
         at(0, 37), (at(0, 39) - at(0, 38)) / 100.0, at(0, 37) / ((at(0, 39) - at(0, 38)) / 100.0), at(0, 1));
  printf("  p | A work: w0 w1 w2 w3 | A sync done | B work: w0 w1 w2 w3 | B sync done\n");
  for (int p = 0; p < 8; ++p) {
    const double start = p == 0 ? at(0, 1) : at(0, 5 + 4 * (p - 1));
    printf("  %d |", p);
    for (int w = 0; w < 4; ++w) printf(" %6.0f", at(w, 2 + 4 * p) - start);
    printf(" | %6.0f |", at(0, 3 + 4 * p) - start);
    for (int w = 0; w < 4; ++w) printf(" %6.0f", at(w, 4 + 4 * p) - at(0, 3 + 4 * p));
    printf(" | %6.0f\n", at(0, 5 + 4 * p) - at(0, 3 + 4 * p));
  }
  printf("  tail T: %.0f  sync %.0f  finish+zeros+drain %.0f\n", at(0, 34) - at(0, 33), at(0, 35) - at(0, 34),
         at(0, 37) - at(0, 35));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int n = 128;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      h[i * n + j] = (i == j ? 4.0 : 0.0) + exp(-0.01 * (i - j) * (i - j)) + 1e-3 * ((i * 7 + j * 7) % 13);
  double *A, *Li, *ld;
  unsigned long long* st;
  CK(hipMalloc(&A, n * n * 8)); CK(hipMalloc(&Li, n * n * 8)); CK(hipMalloc(&ld, n * 8));
  CK(hipMalloc(&st, 4 * NST * 8));
  CK(hipMemcpy(A, h.data(), n * n * 8, hipMemcpyHostToDevice));
  const int which = argc > 2 ? atoi(argv[2]) : 0;
  if (which == 0) {
    probe<0>(A, Li, ld, st, reps);
    probe<1>(A, Li, ld, st, reps);
    probe<2>(A, Li, ld, st, reps);
    probe<4>(A, Li, ld, st, reps);
    probe<8>(A, Li, ld, st, reps);
    probe<7>(A, Li, ld, st, reps);
    probe<15>(A, Li, ld, st, reps);
  } else if (which == 2) {
    probe<0, 0, false>(A, Li, ld, st, reps);
    probe<0, 0, true>(A, Li, ld, st, reps);
    probe<0, 3, true>(A, Li, ld, st, reps);
    probe<0, 4, true>(A, Li, ld, st, reps);
    probe<4, 0, true>(A, Li, ld, st, reps);
    probe<4, 3, true>(A, Li, ld, st, reps);
  } else {
    probe<0>(A, Li, ld, st, reps);
    probe<0, 2>(A, Li, ld, st, reps);
    probe<0, 3>(A, Li, ld, st, reps);
    probe<0, 4>(A, Li, ld, st, reps);
    probe<4, 3>(A, Li, ld, st, reps);
    probe<4, 4>(A, Li, ld, st, reps);
  }
  return 0;
}
