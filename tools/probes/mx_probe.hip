// Probe (GPU): OCP e4m3 conversion and the operand layout of the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 on gfx950, with exact small-integer data.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/mx_probe.hip -o tools/probes/mx_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void cvt_probe(const float* in, uint32_t* out, int n) {
  int i = threadIdx.x;
  if (i < n) out[i] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(in[i], -in[i], 0, false);
}

// A, B given as fp8 bytes in "lane order": lane l supplies bytes a[l*32 .. l*32+31].
__global__ void mfma_probe(const uint8_t* a, const uint8_t* b, float* d, int sa, int sb) {
  const int l = threadIdx.x;
  if (sa < 0) {                     // per-lane scales: A block of lane l scaled by 2^sA(l)
    sa = 127 + ((l >> 4) & 1) + ((l & 15) == 3 ? 2 : 0);
    sb = 127 + ((l >> 5) & 1) + ((l & 15) == 5 ? 1 : 0);
  }
  i32x8 av, bv;
  const int* ap = reinterpret_cast<const int*>(a + l * 32);
  const int* bp = reinterpret_cast<const int*>(b + l * 32);
  for (int i = 0; i < 8; ++i) { av[i] = ap[i]; bv[i] = bp[i]; }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

static uint8_t e4m3(float v) {   // exact for small integers / halves
  if (v == 0) return 0;
  uint8_t s = v < 0 ? 0x80 : 0;
  v = fabsf(v);
  int e = (int)floorf(log2f(v));
  float m = v / ldexpf(1.f, e) - 1.f;
  return s | (uint8_t)((e + 7) << 3) | (uint8_t)lrintf(m * 8);
}

int main() {
  std::vector<float> in = {1.f, 2.f, 0.5f, 3.f, -1.f, 448.f, 0.f, 1.5f};
  float* din; uint32_t* dout;
  hipMalloc(&din, 64); hipMalloc(&dout, 64);
  hipMemcpy(din, in.data(), 32, hipMemcpyHostToDevice);
  cvt_probe<<<1, 64>>>(din, dout, 8);
  uint32_t o[8];
  hipMemcpy(o, dout, 32, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i)
    printf("cvt %g -> lo %02x hi %02x  (OCP e4m3 expects %02x / %02x)\n", in[i], o[i] & 0xff, (o[i] >> 8) & 0xff,
           e4m3(in[i]), e4m3(-in[i]));
  // A[16][128], B[128][16] with small integers.
  std::vector<float> A(16 * 128), B(128 * 16);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) A[i * 128 + k] = (float)(((i * 7 + k * 3) % 5) - 2);
  for (int k = 0; k < 128; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (float)(((k * 5 + j * 11) % 7) - 3) * 0.5f;
  // Hypothesis H1: lane l: row/col l&15, k = 32*(l>>4) + j.
  // Hypothesis H2: lane l: k = 16*(l>>4) + j (j < 16), 64 + 16*(l>>4) + (j - 16) (j >= 16).
  for (int hyp = 1; hyp <= 2; ++hyp) {
    std::vector<uint8_t> ab(64 * 32), bb(64 * 32);
    auto kof = [&](int l, int j) { return hyp == 1 ? 32 * (l >> 4) + j : (j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + j - 16); };
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        ab[l * 32 + j] = e4m3(A[(l & 15) * 128 + kof(l, j)]);
        bb[l * 32 + j] = e4m3(B[kof(l, j) * 16 + (l & 15)]);
      }
    uint8_t *da, *db; float* dd;
    hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dd, 64 * 16);
    hipMemcpy(da, ab.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(db, bb.data(), 2048, hipMemcpyHostToDevice);
    for (int sc = 0; sc < 3; ++sc) {
      const int sa = sc == 2 ? -1 : 127 + sc, sb = 127;      // E8M0: 127 = 2^0
      mfma_probe<<<1, 64>>>(da, db, dd, sa, sb);
      std::vector<float> D(256);
      hipMemcpy(D.data(), dd, 1024, hipMemcpyDeviceToHost);
      double err = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * (l >> 4) + r, col = l & 15;
          double ref = 0;
          for (int k = 0; k < 128; ++k) {
            double f = 1.0;
            if (sc == 2) {
              int lg = -1;                          // lane group holding k (same map for A and B)
              for (int g = 0; g < 4 && lg < 0; ++g)
                for (int j = 0; j < 32; ++j) if (kof(g * 16, j) == k) { lg = g; break; }
              const int ea = (lg & 1) + (row == 3 ? 2 : 0), eb = ((lg >> 1) & 1) + (col == 5 ? 1 : 0);
              f = ldexp(1.0, ea + eb);
            }
            ref += (double)A[row * 128 + k] * B[k * 16 + col] * f;
          }
          ref *= (sc == 1 ? 2.0 : 1.0);
          err = fmax(err, fabs(ref - D[l * 4 + r]));
        }
      printf("hyp %d scale_a=%d: max abs err %g\n", hyp, sa, err);
    }
  }
  return 0;
}
