// Probe: the per-launch cost of dependent kernels inside one hipGraph (the UNet step's 134
// launches run this way): N back-to-back launches of a trivial kernel on one captured stream,
// for several grid sizes; prints us per launch. Also the same N launches issued eagerly.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void tiny(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(buf, 0, 64 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int N = 400;
  for (int blocks : {1, 256, 1024, 4096}) {
    const int n = blocks * 256;
    hipGraph_t g; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) tiny<<<blocks, 256, 0, st>>>(buf, n);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ex, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double graph_us = ms * 1e3 / (5.0 * N);
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r)
      for (int i = 0; i < N; ++i) tiny<<<blocks, 256, 0, st>>>(buf, n);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("blocks %5d: graph %.2f us/launch, eager %.2f us/launch\n", blocks, graph_us, ms * 1e3 / (5.0 * N));
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
  }
  return 0;
}
