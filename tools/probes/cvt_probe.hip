#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short short2_ __attribute__((ext_vector_type(2)));
__global__ void k(unsigned* out) {
  bf16x2 v = {(__bf16)1.0f, (__bf16)3.0f};
  short2_ r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(short2_{0, 0}, v, 2.0f, false);
  short2_ r2 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, v, 0.5f, true);
  out[0] = __builtin_bit_cast(unsigned, r2);
}
int main() {
  unsigned* d; unsigned h = 0;
  (void)hipMalloc(&d, 4);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  // e4m3: 0.5=0x30 1.0=0x38 1.5=0x3c 2.0=0x40 3.0=0x44 6.0=0x4c
  printf("cvt_scalef32_pk_fp8_bf16: %08x (bytes lo..hi)\n", h);
  return 0;
}
