// Probe (GPU): do kernels of two independent branches run concurrently on MI355X — on two
// streams, and inside one hipGraph captured with a fork / join (event record / wait)?
// A "chain" = N launches of a latency-bound kernel (few blocks, a dependent FMA loop), the
// shape of the UNet's 32x32-level kernels. Prints the time of one chain, two chains back to
// back on one stream, two chains on two streams, and the graph of two parallel chains.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/graph_concur.hip -o tools/probes/graph_concur
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void spin(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, 1e-7f);
  if (a == 12345.f) out[blockIdx.x] = a;        // (never true; keeps the loop)
}

int main() {
  float* d;
  CK(hipMalloc(&d, 4096));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, fork, j1;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
  const int N = 50, BLK = 64, IT = 20000;
  auto chain = [&](hipStream_t s) { for (int i = 0; i < N; ++i) spin<<<BLK, 256, 0, s>>>(d, IT); };
  auto timeit = [&](auto fn, hipStream_t s) -> float {
    fn(); (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, s);
    fn();
    (void)hipEventRecord(b, s);
    (void)hipDeviceSynchronize();
    float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
    return ms;
  };
  printf("one chain        %8.3f ms\n", timeit([&] { chain(s0); }, s0));
  printf("two, one stream  %8.3f ms\n", timeit([&] { chain(s0); chain(s0); }, s0));
  // two streams: fork from s0, join back to s0
  printf("two streams      %8.3f ms\n", timeit([&] {
    hipEventRecord(fork, s0); hipStreamWaitEvent(s1, fork, 0); hipStreamWaitEvent(s2, fork, 0);
    chain(s1); chain(s2);
    hipEventRecord(j1, s1); hipStreamWaitEvent(s0, j1, 0); hipEventRecord(j1, s2); hipStreamWaitEvent(s0, j1, 0);
  }, s0));
  // graph with two parallel branches
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  CK(hipEventRecord(fork, s0));
  CK(hipStreamWaitEvent(s1, fork, 0));
  chain(s0); chain(s1);
  CK(hipEventRecord(j1, s1));
  CK(hipStreamWaitEvent(s0, j1, 0));
  CK(hipStreamEndCapture(s0, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  printf("graph, 2 branches %7.3f ms\n", timeit([&] { hipGraphLaunch(ge, s0); }, s0));
  hipGraph_t g1; hipGraphExec_t ge1;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  chain(s0); chain(s0);
  CK(hipStreamEndCapture(s0, &g1));
  CK(hipGraphInstantiate(&ge1, g1, nullptr, nullptr, 0));
  printf("graph, 1 branch   %7.3f ms\n", timeit([&] { hipGraphLaunch(ge1, s0); }, s0));
  return 0;
}
