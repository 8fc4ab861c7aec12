// Dependent-launch latency on one stream: N tiny kernels back to back, plain stream vs
// one captured hipGraph, and with an event record/wait pair between launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void tiny(double* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1.0; }
int main() {
  double* d; hipMalloc(&d, 1024 * 8);
  hipStream_t s, s2; hipStreamCreateWithFlags(&s, hipStreamNonBlocking); hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int N = 1000;
  for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, d);
  hipStreamSynchronize(s);
  float ms;
  hipEventRecord(e0, s);
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, d);
  hipEventRecord(e1, s); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("stream: %.2f us per dependent launch\n", 1e3 * ms / N);
  // with a fork/join through a second stream every 4th launch (like the recursion's side stream)
  hipEvent_t f; hipEventCreateWithFlags(&f, hipEventDisableTiming);
  hipEventRecord(e0, s);
  for (int i = 0; i < N; ++i) {
    hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, d);
    if (i % 4 == 0) { hipEventRecord(f, s); hipStreamWaitEvent(s2, f, 0); hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s2, d + 512); }
  }
  hipEventRecord(e1, s); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("stream + side fork every 4th: %.2f us per main launch\n", 1e3 * ms / N);
  hipStreamSynchronize(s2);
  // graph
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(4), dim3(64), 0, s, d);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s); hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  hipGraphLaunch(ge, s);
  hipEventRecord(e1, s); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("graph: %.2f us per dependent launch\n", 1e3 * ms / N);
  return 0;
}
