// Probe (GPU): which lane's E8M0 scale applies to which lane's operand block in
// v_mfma_scale_f32_16x16x128_f8f6f4. Block (L, S, which): A (which=0) or B (which=1) is 1.0
// only in lane L's 32 bytes (the other operand all 1.0); lane S's scale is 2^1, all others 2^0.
// out[which][L][S] = sum of D / 512 (1 or 2).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out) {
  const int L = blockIdx.x, S = blockIdx.y, which = blockIdx.z, l = threadIdx.x;
  const int one = 0x38383838;           // four e4m3 1.0
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (which == 1 || l == L) ? one : 0;
    b[i] = (which == 0 || l == L) ? one : 0;
  }
  const int sa = (which == 0 && l == S) ? 128 : 127;
  const int sb = (which == 1 && l == S) ? 128 : 127;
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  float s = c[0] + c[1] + c[2] + c[3];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (l == 0) out[(which * 64 + L) * 64 + S] = s / 512.f;
}
int main() {
  float* d;
  (void)hipMalloc(&d, 2 * 64 * 64 * 4);
  probe<<<dim3(64, 64, 2), 64>>>(d);
  static float h[2 * 64 * 64];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int w = 0; w < 2; ++w)
    for (int L = 0; L < 64; ++L) {
      printf("%c data lane %2d: scale lanes", w ? 'B' : 'A', L);
      for (int S = 0; S < 64; ++S) if (h[(w * 64 + L) * 64 + S] > 1.01f) printf(" %d:%.3g", S, h[(w * 64 + L) * 64 + S]);
      printf("\n");
    }
  return 0;
}
