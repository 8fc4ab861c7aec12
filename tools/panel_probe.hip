// Probe (not in the library): cycles for ONE wave to factor a 128×16 Cholesky panel held in
// registers (lane l: rows l and l+64), pivots and multipliers broadcast by v_readlane — the
// pivot-wave step of the MFMA leaf design.  Prints cycles per panel (s_memtime = shader clock).
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rl(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// variant 1: straightforward; variant 2: diagonal-tile slot known at compile time (DS), slot 0
// skipped when it holds no panel row (LO = false), next pivot's chain first
template <int DS, bool LO>
__device__ __forceinline__ void factor_panel(double (&P)[2][16], int J0, int l) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j, lJ = J & 63;
    const double d = rl(P[DS][j], lJ);
    const double rs = __builtin_amdgcn_rsq(d);
    const double ljj = d * rs;
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) {
      const int R = l + 64 * s;
      const double v = P[s][j] * rs;
      P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
    }
#pragma unroll
    for (int c = j + 1; c < 16; ++c) {
      const double m = rl(P[DS][j], (J0 + c) & 63);
#pragma unroll
      for (int s = LO ? 0 : 1; s < 2; ++s) P[s][c] = fma(-P[s][j], m, P[s][c]);
    }
  }
}

// variant 3/4: multipliers of column j published once to LDS by the lanes holding them and
// read back as broadcasts (ds_read_b128 pairs); variant 4 takes the next pivot's multiplier
// (the dependent chain) by v_readlane instead
template <int DS, bool LO, bool RL1, int RSQ = 0, bool EXTRA = false>
__device__ __forceinline__ void factor_panel_lds(double (&P)[2][16], int J0, int l, double* M,
                                                 double* DG = nullptr, int* badp = nullptr) {
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j, lJ = J & 63;
    const double d = rl(P[DS][j], lJ);
    double rs;
    if (RSQ == 0) rs = __builtin_amdgcn_rsq(d);
    else if (RSQ == 1) rs = rsqrt(d);
    else { const double y = __builtin_amdgcn_rsq(d); rs = y * fma(-0.5 * d * y, y, 1.5); }
    if (EXTRA) {
      if (!(d > 0.0) && J < 1000 && bad == 0) bad = J + 1;
    }
    const double ljj = d * rs;
    if (EXTRA && l == 0) { DG[J] = ljj; DG[128 + J] = rs; }
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) {
      const int R = l + 64 * s;
      const double v = P[s][j] * rs;
      P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
    }
    double* Mj = M + 16 * (j & 1);  // double-buffered so a lagging read never sees column j+1
    {
      const int R = l + 64 * DS;
      if (R > J && R < J0 + 16) Mj[R - J0] = P[DS][j];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double m1 = 0.0;
    if (RL1 && j < 15) m1 = rl(P[DS][j], (J + 1) & 63);
#pragma unroll
    for (int c = j + 1; c < 16; ++c) {
      const double m = (RL1 && c == j + 1) ? m1 : Mj[c];
#pragma unroll
      for (int s = LO ? 0 : 1; s < 2; ++s) P[s][c] = fma(-P[s][j], m, P[s][c]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  if (EXTRA && badp) *badp = bad;
}

// variant 7: the diagonal tile's column j replicated to all four 16-lane rows by ds_bpermute
// (two per column), then each multiplier L[J0+c][j] taken by a 64-bit DPP row_newbcast:c of that
// copy — no v_readlane pair (and its SGPR hazards) per multiplier; the chain's next pivot column
// (c = j+1) keeps its v_readlane.  Same FMAs in the same order per element: bitwise equal to v2.
template <int C>
__device__ __forceinline__ double nbcast(double x) {
  long long v = __double_as_longlong(x), old = 0;
  long long r = __builtin_amdgcn_update_dpp(old, v, 0x150 + C, 0xf, 0xf, true);
  return __longlong_as_double(r);
}
template <int DS, bool LO>
__device__ __forceinline__ void factor_panel_dpp(double (&P)[2][16], int J0, int l) {
  const int src = 4 * ((J0 & 63) + (l & 15));  // bpermute byte address: the diagonal row's lane
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j, lJ = J & 63;
    const double d = rl(P[DS][j], lJ);
    const double y = __builtin_amdgcn_rsq(d);
    const double rs = y * fma(-0.5 * d * y, y, 1.5);
    const double ljj = d * rs;
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) {
      const int R = l + 64 * s;
      const double v = P[s][j] * rs;
      P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
    }
    if (j == 15) break;
    const double pj = P[DS][j];
    const int lo = __builtin_amdgcn_ds_bpermute(src, __double2loint(pj));
    const int hi = __builtin_amdgcn_ds_bpermute(src, __double2hiint(pj));
    const double m1 = rl(pj, (J + 1) & 63);
#pragma unroll
    for (int s = LO ? 0 : 1; s < 2; ++s) P[s][j + 1] = fma(-P[s][j], m1, P[s][j + 1]);
    const double Mrep = __hiloint2double(hi, lo);
#define GPS_UPD(C)                                                                     \
    if (C > j + 1) {                                                                   \
      const double m = nbcast<C>(Mrep);                                                \
      _Pragma("unroll") for (int s = LO ? 0 : 1; s < 2; ++s) P[s][C] = fma(-P[s][j], m, P[s][C]); \
    }
    GPS_UPD(2) GPS_UPD(3) GPS_UPD(4) GPS_UPD(5) GPS_UPD(6) GPS_UPD(7) GPS_UPD(8) GPS_UPD(9)
    GPS_UPD(10) GPS_UPD(11) GPS_UPD(12) GPS_UPD(13) GPS_UPD(14) GPS_UPD(15)
#undef GPS_UPD
  }
}

// variant 8: the library's factor_panel as built (csrc/kernels_potrf.hip v4::factor_panel:
// v_readlane multipliers, v_rsq_f64 + one Newton step, wave barriers between the phases)
template <int DS, bool LO>
__device__ __forceinline__ void factor_panel_lib(double (&P)[2][16], int J0, int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int J = J0 + j;
    const double d = rl(P[DS][j], J & 63);
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

template <int V>
__global__ __launch_bounds__(64) void panel_kernel(const double* in, double* out, long long* cyc, int p) {
  const int l = threadIdx.x;
  double P[2][16];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 16; ++c) P[s][c] = in[(l + 64 * s) * 16 + c];
  const int J0 = 16 * p;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(P[s][c]));
  long long t0, r0, t1, r1;
  asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(P[s][c]) : "s"(t0));
  if (V == 1) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int J = J0 + j, sJ = J >> 6, lJ = J & 63;
      const double d = rl(sJ ? P[1][j] : P[0][j], lJ);
      const double rs = __builtin_amdgcn_rsq(d);
      const double ljj = d * rs;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R = l + 64 * s;
        const double v = P[s][j] * rs;
        P[s][j] = R > J ? v : (R == J ? ljj : 0.0);
      }
#pragma unroll
      for (int c = j + 1; c < 16; ++c) {
        const int C = J0 + c;
        const double m = rl((C >> 6) ? P[1][j] : P[0][j], C & 63);
#pragma unroll
        for (int s = 0; s < 2; ++s) P[s][c] = fma(-P[s][j], m, P[s][c]);
      }
    }
  } else if (V == 2) {
    if (p < 4) factor_panel<0, true>(P, J0, l);
    else factor_panel<1, false>(P, J0, l);
  } else if (V == 8) {
    if (p < 4) factor_panel_lib<0, true>(P, J0, l);
    else factor_panel_lib<1, false>(P, J0, l);
  } else if (V == 7) {
    if (p < 4) factor_panel_dpp<0, true>(P, J0, l);
    else factor_panel_dpp<1, false>(P, J0, l);
  } else if (V <= 4) {
    __shared__ double M[32];
    if (p < 4) factor_panel_lds<0, true, V == 4>(P, J0, l, M);
    else factor_panel_lds<1, false, V == 4>(P, J0, l, M);
  } else {
    __shared__ double M[32];
    __shared__ double DG[256];
    __shared__ int badv;
    constexpr int RSQ = V == 5 ? 1 : 2;
    if (p < 4) factor_panel_lds<0, true, true, RSQ, true>(P, J0, l, M, DG, &badv);
    else factor_panel_lds<1, false, true, RSQ, true>(P, J0, l, M, DG, &badv);
    if (l == 0) cyc[2] = badv + (long long)DG[J0];
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(P[s][c]));
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_nop 7\n s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 16; ++c) out[(l + 64 * s) * 16 + c] = P[s][c];
  if (l == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

int main() {
  double h[128 * 16];
  for (int r = 0; r < 128; ++r)
    for (int c = 0; c < 16; ++c) h[r * 16 + c] = (r % 16 == c) ? 64.0 : 0.01 * ((r * 7 + c * 3) % 11 - 5);
  double *in, *out; long long* cyc;
  (void)hipMalloc(&in, sizeof(h)); (void)hipMalloc(&out, sizeof(h)); (void)hipMalloc(&cyc, 24);
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int v : {8, 7})
    for (int p : {0, 3, 4, 7}) {
      long long best[2] = {1ll << 60, 0};
      for (int rep = 0; rep < 20; ++rep) {
        if (v == 1) panel_kernel<1><<<1, 64>>>(in, out, cyc, p);
        else if (v == 2) panel_kernel<2><<<1, 64>>>(in, out, cyc, p);
        else if (v == 3) panel_kernel<3><<<1, 64>>>(in, out, cyc, p);
        else if (v == 4) panel_kernel<4><<<1, 64>>>(in, out, cyc, p);
        else if (v == 5) panel_kernel<5><<<1, 64>>>(in, out, cyc, p);
        else if (v == 7) panel_kernel<7><<<1, 64>>>(in, out, cyc, p);
        else if (v == 8) panel_kernel<8><<<1, 64>>>(in, out, cyc, p);
        else panel_kernel<6><<<1, 64>>>(in, out, cyc, p);
        long long c[2]; (void)hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
        if (c[0] < best[0]) { best[0] = c[0]; best[1] = c[1]; }
      }
      static double ref[4][128 * 16];
      double o[128 * 16];
      (void)hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
      const int pi = p == 0 ? 0 : p == 3 ? 1 : p == 4 ? 2 : 3;
      double err = 0.0;
      for (int i = 0; i < 128 * 16; ++i) {
        if (i / 16 < 16 * p) continue;  // rows above the panel's diagonal tile: unused
        if (v == 8) ref[pi][i] = o[i];
        else err = fmax(err, fabs(o[i] - ref[pi][i]));
      }
      printf("variant %d panel p=%d: %lld cycles (%lld ns)  max|diff vs v8| %.1e\n", v, p, best[0], best[1] * 10, err);
    }
  return 0;
}
