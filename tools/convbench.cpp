// Standalone microbenchmark of the conv kernels (links da-clip_amd/build/conv*.o).
// Usage: convbench [iters]   — prints per-shape time and TFLOP/s for bf16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../da-clip_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
using namespace dac;
typedef __bf16 bf16;

struct Shape { const char* name; int B, H, W, cin, cout, kh, s, p, up, act, ss, res; };

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;   // substring filter on the shape name
  std::vector<Shape> shapes = {
    {"L0 3x3 64->64 plain", 8, 256, 256, 64, 64, 3, 1, 1, 0, 0, 0, 0},
    {"L0 3x3 64->64 ss+silu", 8, 256, 256, 64, 64, 3, 1, 1, 0, 1, 1, 0},
    {"L0 3x3 64->64 silu+res", 8, 256, 256, 64, 64, 3, 1, 1, 0, 1, 0, 1},
    {"L0 3x3 128->64 ss+silu", 8, 256, 256, 128, 64, 3, 1, 1, 0, 1, 1, 0},
    {"L1 3x3 192->128", 8, 128, 128, 192, 128, 3, 1, 1, 0, 1, 1, 0},
    {"L2 3x3 256->256", 8, 64, 64, 256, 256, 3, 1, 1, 0, 1, 1, 0},
    {"L3 3x3 512->512", 8, 32, 32, 512, 512, 3, 1, 1, 0, 1, 1, 0},
    {"L0 1x1 64->384", 8, 256, 256, 64, 384, 1, 1, 0, 0, 0, 0, 0},
    {"L0 1x1 128->64", 8, 256, 256, 128, 64, 1, 1, 0, 0, 0, 0, 0},
    {"L3 1x1 512->4096", 8, 32, 32, 512, 4096, 1, 1, 0, 0, 0, 0, 0},
  };
  size_t maxe = (size_t)8 * 256 * 256 * 512;
  void *x, *y, *w, *res, *zero; float *ss, *bias;
  CK(hipMalloc(&x, maxe * 2)); CK(hipMalloc(&y, maxe * 2)); CK(hipMalloc(&res, maxe * 2));
  CK(hipMalloc(&w, (size_t)4096 * 9 * 1024 * 2)); CK(hipMalloc(&zero, 256));
  CK(hipMalloc(&ss, 8 * 8192 * 4)); CK(hipMalloc(&bias, 8192 * 4));
  CK(hipMemset(zero, 0, 256)); CK(hipMemset(x, 0x3c, maxe * 2)); CK(hipMemset(w, 0x3c, (size_t)4096 * 9 * 1024 * 2));
  CK(hipMemset(ss, 0, 8 * 8192 * 4)); CK(hipMemset(res, 0, maxe * 2));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& s : shapes) {
    if (only && !strstr(s.name, only)) continue;
    ConvArgs a{};
    a.x1 = x; a.ld1 = s.cin; a.C1 = s.cin; a.Cin = s.cin; a.Hs = s.H; a.Ws = s.W; a.up = s.up;
    a.B = s.B; a.Ho = (s.H + 2 * s.p - s.kh) / s.s + 1; a.Wo = (s.W + 2 * s.p - s.kh) / s.s + 1;
    a.Cout = s.cout; a.K = s.kh * s.kh * s.cin; a.w = w; a.y = y; a.ldy = s.cout; a.act = s.act;
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
    printf("%-26s variant %d  %8.1f us  %7.1f TF/s  %6.0f GB/s(min bytes)\n", s.name,
           conv_variant(a, s.kh, 2), us, fl / us / 1e6, by / us / 1e3);
  }
  return 0;
}
