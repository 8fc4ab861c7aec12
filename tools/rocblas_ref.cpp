// Reference point only (never linked into the product): rocBLAS DGEMM / DSYRK / DTRMM throughput
// on the shapes of the C3 recursion's top level, to see how close gemm_f64_kernel is to the
// vendor library on this chip.  Build: see tools/run_rocblas_ref.sh.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdio.h>
#include <vector>
__global__ void fill(double* p, size_t n, unsigned long long s) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long x = (i + 1) * 6364136223846793005ull + s;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
    p[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}
int main() {
  rocblas_handle h; rocblas_create_handle(&h);
  const int n = 10112;
  double *A, *B, *C;
  hipMalloc(&A, (size_t)n * n * 8); hipMalloc(&B, (size_t)n * n * 8); hipMalloc(&C, (size_t)n * n * 8);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, (size_t)n * n, 1ull);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, B, (size_t)n * n, 2ull);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, C, (size_t)n * n, 3ull);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double one = 1.0, mone = -1.0;
  auto timeit = [&](const char* name, double flops, auto fn) {
    fn(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) fn();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.3f ms  %6.2f TF/s\n", name, ms / 3, flops / (ms / 3 * 1e-3) / 1e12);
  };
  timeit("dgemm NT 10112^3", 2.0 * n * n * (double)n, [&] {
    rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, n, n, n, &one, B, n, A, n, &one, C, n); });
  timeit("dgemm NN 8192^3", 2.0 * 8192.0 * 8192 * 8192, [&] {
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, 8192, 8192, 8192, &one, A, 8192, B, 8192, &one, C, 8192); });
  timeit("dsyrk lower 10112 K=9984", (double)n * (n + 1) * 9984, [&] {
    rocblas_dsyrk(h, rocblas_fill_upper, rocblas_operation_transpose, n, 9984, &mone, A, 9984, &one, C, n); });
  timeit("dtrmm 10112x9984 (tri 10112)", (double)n * n * 9984, [&] {
    rocblas_dtrmm(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit,
                  n, 9984, &one, A, n, B, n, C, n); });
  rocblas_destroy_handle(h);
  return 0;
}
