// Ablation timing of the 128×128 diagonal-block kernel (potrf + inverse).
// Built four times with GPS_DIAG_ABLATE = 0..3 by tools/run_diag_bench.sh.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#include "kernels_potrf.hip"
using namespace gps;
int main() {
  const int n = 128;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
  double *A, *Li, *ld; int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&Li, n * n * 8); hipMalloc(&ld, n * 8); hipMalloc(&info, 4);
  hipMemcpy(A, h.data(), n * n * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) launch_potrf_diag(A, n, Li, n, nullptr, 0, ld, info, 0, n, 0);
  const int reps = 200;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) launch_potrf_diag(A, n, Li, n, nullptr, 0, ld, info, 0, n, 0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("ablate=%d  %.2f us per diag block\n", GPS_DIAG_ABLATE, 1e3 * ms / reps);
#ifdef GPS_DIAG_STAMPS
  std::vector<unsigned long long> st(32 * 8 * 17);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(gps_stamps), st.size() * 8);
  // per step: owner pivot (slot1-slot0 of the owner), barrier1 wait (max over waves of 2-1),
  // panel (3-2), barrier2 (4-3), rest of step (next 0 - 4)
  double sp = 0, sb1 = 0, spn = 0, sb2 = 0, st_ = 0;
  for (int jb = 0; jb < 32; ++jb) {
    auto S = [&](int slot, int w) { return (double)st[(jb * 8 + slot) * 17 + w]; };
    double piv = S(1, 16) - S(0, 16);
    double t0 = 1e30, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    for (int w = 0; w < 16; ++w) { t0 = std::min(t0, S(0, w)); t1 = std::max(t1, S(1, w)); t2 = std::max(t2, S(2, w)); t3 = std::max(t3, S(3, w)); t4 = std::max(t4, S(4, w)); }
    double next = jb < 31 ? 1e30 : t4;
    if (jb < 31) for (int w = 0; w < 16; ++w) next = std::min(next, (double)st[((jb + 1) * 8 + 0) * 17 + w]);
    if (jb < 4 || jb == 16 || jb == 30)
      printf("jb=%2d pivot(owner)=%6.0f  t0->allarrive1=%6.0f  bar1->allarrive3=%6.0f  ->allarrive4=%6.0f  ->next=%6.0f\n",
             jb, piv, t1 - t0, t3 - t2, t4 - t3, next - t4);
    sp += piv; sb1 += t1 - t0; spn += t3 - t2; sb2 += t4 - t3; st_ += next - t4;
  }
  printf("sum cycles: pivot %.0f  phaseA %.0f  panel %.0f  bar2 %.0f  trailing %.0f\n", sp, sb1, spn, sb2, st_);
#endif
  return 0;
}
