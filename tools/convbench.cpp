// Standalone microbenchmark of the conv kernels (links da-clip_amd/build/conv*.o).
// Usage: convbench [iters] [shape-substring] [check|-] [force-list]
//   force-list: comma-separated 3x3 kernel choices (-1 built-in, 0 v3, k>0 v4 config k)
//   prints per-shape time and TFLOP/s for bf16; with "check" the inputs are random and every
//   output is compared with a naive reference conv (fp32 accumulate, same epilogue).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
#include "../da-clip_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
using namespace dac;
extern "C" void dac_conv3_force(int v);
extern "C" void dac_conv2_force(int v);
typedef __bf16 bf16;

struct Shape { const char* name; int B, H, W, cin, cout, kh, s, p, up, act, ss, res, kwp = 0, bias = 0; };

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed, float scale) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed;
  h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
  p[i] = (bf16)(((h & 0xffff) / 65535.f - 0.5f) * scale);
}
__global__ void fill_rand_f(float* p, size_t n, uint32_t seed, float scale) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed;
  h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
  p[i] = ((h & 0xffff) / 65535.f - 0.5f) * scale;
}
// Naive reference: one thread per output element; weights [Cout][kh][kw][Cin].
__global__ void ref_conv(ConvArgs a, int kh, int s, int p, int kws, float* out) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t M = (size_t)a.B * a.Ho * a.Wo;
  if (i >= M * a.Cout) return;
  const int n = i % a.Cout;
  const size_t m = i / a.Cout;
  const int b = m / (a.Ho * a.Wo), r = m % (a.Ho * a.Wo), oh = r / a.Wo, ow = r % a.Wo;
  const bf16* x = (const bf16*)a.x1;
  const bf16* w = (const bf16*)a.w;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  float acc = 0.f;
  for (int y = 0; y < kh; ++y)
    for (int z = 0; z < kh; ++z) {
      const int ih = oh * s - p + y, iw = ow * s - p + z;
      if (ih < 0 || iw < 0 || ih >= Hin || iw >= Win) continue;
      const int sh = a.up ? ih >> 1 : ih, sw = a.up ? iw >> 1 : iw;
      const bf16* xp = x + ((size_t)(b * a.Hs + sh) * a.Ws + sw) * a.ld1;
      const bf16* wp = w + (((size_t)n * kh + y) * kws + z) * a.Cin;
      for (int c = 0; c < a.Cin; ++c) acc += (float)xp[c] * (float)wp[c];
    }
  if (a.bias) acc += a.bias[n];
  if (a.ss) acc = acc * (a.ss[(size_t)b * a.ss_ld + n] + 1.f) + a.ss[(size_t)b * a.ss_ld + a.Cout + n];
  if (a.act == 1) acc = acc / (1.f + expf(-acc));
  if (a.res1) acc += (float)((const bf16*)a.res1)[m * a.ldr1 + n];
  out[i] = acc;
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20;
  const char* only = argc > 2 && argv[2][0] ? argv[2] : nullptr;   // substring filter
  const bool check = argc > 3 && !strcmp(argv[3], "check");
  std::vector<int> forces;
  if (argc > 4) {
    for (char* t = strtok(argv[4], ","); t; t = strtok(nullptr, ",")) forces.push_back(atoi(t));
  } else forces.push_back(-1);
  std::vector<Shape> shapes = {
    {"L0 3x3 64->64 plain", 8, 256, 256, 64, 64, 3, 1, 1, 0, 0, 0, 0},
    {"L0 3x3 64->64 ss+silu", 8, 256, 256, 64, 64, 3, 1, 1, 0, 1, 1, 0},
    {"L0 3x3 64->64 silu+res", 8, 256, 256, 64, 64, 3, 1, 1, 0, 1, 0, 1},
    {"L0 3x3 128->64 ss+silu", 8, 256, 256, 128, 64, 3, 1, 1, 0, 1, 1, 0},
    {"L1 3x3 192->128", 8, 128, 128, 192, 128, 3, 1, 1, 0, 1, 1, 0},
    {"L2 3x3 256->256", 8, 64, 64, 256, 256, 3, 1, 1, 0, 1, 1, 0},
    {"L3 3x3 512->512", 8, 32, 32, 512, 512, 3, 1, 1, 0, 1, 1, 0},
    {"L3 3x3 768->512", 8, 32, 32, 768, 512, 3, 1, 1, 0, 1, 1, 0},
    {"L3 3x3 256->256", 8, 32, 32, 256, 256, 3, 1, 1, 0, 1, 1, 0},
    {"L0 1x1 64->384", 8, 256, 256, 64, 384, 1, 1, 0, 0, 0, 0, 0},
    {"L0 1x1 128->64", 8, 256, 256, 128, 64, 1, 1, 0, 0, 0, 0, 0},
    {"L1 1x1 64->384", 8, 128, 128, 64, 384, 1, 1, 0, 0, 0, 0, 0},
    {"L1 1x1 128->384", 8, 128, 128, 128, 384, 1, 1, 0, 0, 0, 0, 0},
    {"L2 1x1 256->384", 8, 64, 64, 256, 384, 1, 1, 0, 0, 0, 0, 0},
    {"L1 3x3 64->64", 8, 128, 128, 64, 64, 3, 1, 1, 0, 1, 1, 0},
    {"L1 3x3 128->128", 8, 128, 128, 128, 128, 3, 1, 1, 0, 1, 1, 0},
    {"L3 1x1 512->4096", 8, 32, 32, 512, 4096, 1, 1, 0, 0, 0, 0, 0},
    {"L3 1x1 512->4096 geglu", 8, 32, 32, 512, 4096, 1, 1, 0, 0, 3, 0, 0, 0, 1},
    {"L3 1x1 256->2048 geglu", 8, 32, 32, 256, 2048, 1, 1, 0, 0, 3, 0, 0, 0, 1},
    {"L3 1x1 512->1536", 8, 32, 32, 512, 1536, 1, 1, 0, 0, 0, 0, 0},
    {"L3 1x1 2048->512 +r", 8, 32, 32, 2048, 512, 1, 1, 0, 0, 0, 0, 1},
    {"L3 1x1 512->512 +r", 8, 32, 32, 512, 512, 1, 1, 0, 0, 0, 0, 1},
    {"L3 1x1 256->256", 8, 32, 32, 256, 256, 1, 1, 0, 0, 0, 0, 0},
    {"L3 1x1 768->512", 8, 32, 32, 768, 512, 1, 1, 0, 0, 0, 0, 0},
    {"L0 7x7 8->64 init", 8, 256, 256, 8, 64, 7, 1, 3, 0, 0, 0, 0, 8},
    {"L0 7x7 8->64 init v1", 8, 256, 256, 8, 64, 7, 1, 3, 0, 0, 0, 0, 0},
    {"L0 3x3 64->3 final", 8, 256, 256, 64, 3, 3, 1, 1, 0, 0, 0, 0, 0, 1},
  };
  size_t maxe = (size_t)8 * 256 * 256 * 512;
  void *x, *y, *w, *res, *zero; float *ss, *bias;
  CK(hipMalloc(&x, maxe * 2)); CK(hipMalloc(&y, maxe * 2)); CK(hipMalloc(&res, maxe * 2));
  CK(hipMalloc(&w, (size_t)4096 * 9 * 1024 * 2)); CK(hipMalloc(&zero, 256));
  CK(hipMalloc(&ss, 8 * 8192 * 4)); CK(hipMalloc(&bias, 8192 * 4));
  CK(hipMemset(zero, 0, 256)); CK(hipMemset(x, 0x3c, maxe * 2)); CK(hipMemset(w, 0x3c, (size_t)4096 * 9 * 1024 * 2));
  CK(hipMemset(ss, 0, 8 * 8192 * 4)); CK(hipMemset(res, 0, maxe * 2)); CK(hipMemset(bias, 0, 8192 * 4));
  float* refo = nullptr;
  bf16* yh = nullptr;
  if (check) {
    const size_t nw = (size_t)4096 * 9 * 1024;
    fill_rand<<<(maxe + 255) / 256, 256>>>((bf16*)x, maxe, 1, 2.f);
    fill_rand<<<(nw + 255) / 256, 256>>>((bf16*)w, nw, 2, 0.1f);
    fill_rand<<<(maxe + 255) / 256, 256>>>((bf16*)res, maxe, 3, 2.f);
    fill_rand_f<<<(8 * 8192 + 255) / 256, 256>>>(ss, 8 * 8192, 4, 1.f);
    fill_rand_f<<<(8192 + 255) / 256, 256>>>(bias, 8192, 5, 1.f);
    CK(hipMalloc(&refo, maxe * 4));
    yh = (bf16*)malloc(maxe * 2);
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& s : shapes) for (int force : forces) {
    if (only && !strstr(s.name, only)) continue;
    // force >= 100: 1x1 (v2) configuration force - 100; otherwise the 3x3 choice.
    dac_conv3_force(force >= 100 ? -1 : force);
    dac_conv2_force(force >= 100 ? force - 100 : 0);
    ConvArgs a{};
    a.x1 = x; a.ld1 = s.cin; a.C1 = s.cin; a.Cin = s.cin; a.Hs = s.H; a.Ws = s.W; a.up = s.up;
    a.B = s.B; a.Ho = (s.H + 2 * s.p - s.kh) / s.s + 1; a.Wo = (s.W + 2 * s.p - s.kh) / s.s + 1;
    const int kws = s.kwp ? s.kwp : s.kh;
    a.Cout = s.cout; a.K = s.kh * kws * s.cin; a.w = w; a.y = y; a.ldy = s.cout < 8 ? 4 : (s.act == 3 ? s.cout / 2 : s.cout); a.act = s.act;
    if (s.bias) a.bias = bias;
    a.zero = zero;
    if (s.ss) { a.ss = ss; a.ss_ld = 2 * s.cout; }
    if (s.res) { a.res1 = res; a.ldr1 = s.cout; }
    for (int i = 0; i < 3; ++i) conv<bf16>(a, s.kh, s.kh, s.s, s.p, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) conv<bf16>(a, s.kh, s.kh, s.s, s.p, 0);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double us = ms * 1e3 / iters;
    double fl = 2.0 * s.B * a.Ho * a.Wo * s.cout * s.kh * s.kh * s.cin;
    double by = 2.0 * ((double)s.B * s.H * s.W * s.cin + (double)s.B * a.Ho * a.Wo * s.cout * (1 + s.res));
    printf("%-26s f%-3d variant %d  %8.1f us  %7.1f TF/s  %6.0f GB/s(min bytes)", s.name, force,
           conv_variant(a, s.kh, 2), us, fl / us / 1e6, by / us / 1e3);
    if (check) {
      const size_t n = (size_t)s.B * a.Ho * a.Wo * s.cout;
      ref_conv<<<(n + 255) / 256, 256>>>(a, s.kh, s.s, s.p, kws, refo);
      CK(hipDeviceSynchronize());
      std::vector<float> r(n);
      CK(hipMemcpy(r.data(), refo, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(yh, y, n / s.cout * a.ldy * 2, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < n; ++i) {
        const size_t yi = (i / s.cout) * a.ldy + i % s.cout;
        md = fmax(md, fabs((double)(float)yh[yi] - r[i]));
        mx = fmax(mx, fabs((double)r[i]));
      }
      printf("  check rel %.2e %s", md / mx, md / mx < 1e-2 ? "OK" : "FAIL");
    }
    printf("\n");
  }
  return 0;
}
