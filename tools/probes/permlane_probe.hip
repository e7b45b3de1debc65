// Probe of v_permlane16/32_swap semantics (common.h red16_* / red32_*): prints, per lane,
// the two swap results for x = lane id.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned x = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(x, x + 100, false, false);
  out[threadIdx.x * 6 + 0] = a[0]; out[threadIdx.x * 6 + 1] = a[1];
  out[threadIdx.x * 6 + 2] = b[0]; out[threadIdx.x * 6 + 3] = b[1];
  out[threadIdx.x * 6 + 4] = c[0]; out[threadIdx.x * 6 + 5] = c[1];
}
int main() {
  unsigned* d; unsigned h[64 * 6];
  (void)hipMalloc(&d, sizeof h);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: p16 %3u %3u  p32 %3u %3u  p16(x,x+100) %3u %3u\n", l, h[l*6], h[l*6+1], h[l*6+2], h[l*6+3], h[l*6+4], h[l*6+5]);
  return 0;
}
