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
#include <algorithm>
#include "../da-clip_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
using namespace dac;
extern "C" void dac_conv3_force(int v);
extern "C" void dac_conv2_force(int v);
extern "C" void dac_conv3r_enable(int on);
extern "C" void dac_rbfuse_enable(int on);
typedef __bf16 bf16;
typedef _Float16 f16;

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
template <typename E> __global__ void ref_conv(ConvArgs a, int kh, int s, int p, int kws, float* out) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t M = (size_t)a.B * a.Ho * a.Wo;
  if (i >= M * a.Cout) return;
  const int n = i % a.Cout;
  const size_t m = i / a.Cout;
  const int b = m / (a.Ho * a.Wo), r = m % (a.Ho * a.Wo), oh = r / a.Wo, ow = r % a.Wo;
  const E* x = (const E*)a.x1;
  const E* w = (const E*)a.w;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  float acc = 0.f;
  for (int y = 0; y < kh; ++y)
    for (int z = 0; z < kh; ++z) {
      const int ih = oh * s - p + y, iw = ow * s - p + z;
      if (ih < 0 || iw < 0 || ih >= Hin || iw >= Win) continue;
      const int sh = a.up ? ih >> 1 : ih, sw = a.up ? iw >> 1 : iw;
      const E* xp = x + ((size_t)(b * a.Hs + sh) * a.Ws + sw) * a.ld1;
      const E* wp = w + (((size_t)n * kh + y) * kws + z) * a.Cin;
      for (int c = 0; c < a.Cin; ++c) acc += (float)xp[c] * (float)wp[c];
    }
  if (a.bias) acc += a.bias[n];
  if (a.ss) acc = acc * (a.ss[(size_t)b * a.ss_ld + n] + 1.f) + a.ss[(size_t)b * a.ss_ld + a.Cout + n];
  if (a.act == 1) acc = acc / (1.f + expf(-acc));
  if (a.res1) acc += (float)((const E*)a.res1)[m * a.ldr1 + n];
  out[i] = acc;
}

// ---- fp8 (conv8.hip) check: host e4m3 quantization identical in spirit to engine.cpp.
static uint8_t f2e4m3(float f) {
  const uint8_t sign = std::signbit(f) ? 0x80 : 0;
  const float a = std::fabs(f);
  if (std::isnan(a)) return 0x7f;
  if (a >= 464.f) return sign | 0x7e;
  if (a < std::ldexp(1.f, -6)) { const int q = (int)std::nearbyint(a * 512.f); return sign | (uint8_t)(q >= 8 ? 8 : q); }
  int e; std::frexp(a, &e);
  int E = e - 1 + 7, q = (int)std::nearbyint((a / std::ldexp(1.f, e - 1) - 1.f) * 8.f);
  if (q == 8) { q = 0; ++E; }
  if (E > 15 || (E == 15 && q == 7)) return sign | 0x7e;
  return sign | (uint8_t)(E << 3) | (uint8_t)q;
}
static float e4m3f(uint8_t b) {
  const int s = b >> 7, E = (b >> 3) & 15, q = b & 7;
  const float v = E ? std::ldexp(1.f + q / 8.f, E - 7) : std::ldexp(q / 8.f, -6);
  return s ? -v : v;
}
static float bf2f(bf16 v) { return (float)v; }
static float bf2f(f16 v) { return (float)v; }
// Quantize rows of n values in 64-blocks: returns dequantized values (and e4m3 bytes + E8M0).
static void quant_rows(const std::vector<float>& v, int rows, int n, int np, std::vector<float>& deq,
                       std::vector<uint8_t>* q8, std::vector<uint8_t>* s8) {
  deq.assign((size_t)rows * n, 0.f);
  if (q8) { q8->assign((size_t)rows * np, 0); s8->assign((size_t)rows * (np / 64), 127); }
  for (int r = 0; r < rows; ++r)
    for (int b = 0; b * 64 < n; ++b) {
      float mx = 0.f;
      for (int k = 64 * b; k < std::min(n, 64 * b + 64); ++k) mx = std::max(mx, std::fabs(v[(size_t)r * n + k]));
      int e = mx > 0.f ? (int)std::ceil(std::log2(mx / 448.f)) : 0;
      e = std::min(126, std::max(-126, e));
      if (s8) (*s8)[(size_t)r * (np / 64) + b] = (uint8_t)(127 + e);
      for (int k = 64 * b; k < std::min(n, 64 * b + 64); ++k) {
        const uint8_t q = f2e4m3(v[(size_t)r * n + k] * std::ldexp(1.f, -e));
        if (q8) (*q8)[(size_t)r * np + k] = q;
        deq[(size_t)r * n + k] = e4m3f(q) * std::ldexp(1.f, e);
      }
    }
}
// Host direct conv (NHWC x [B][H][W][Cin], w [Cout][kh][kw][Cin]) for the fp8 check.
static void host_conv(const std::vector<float>& x, const std::vector<float>& w, int B, int H, int W, int Cin,
                      int Cout, int k, int s, int p, std::vector<float>& y, int& Ho, int& Wo) {
  Ho = (H + 2 * p - k) / s + 1; Wo = (W + 2 * p - k) / s + 1;
  y.assign((size_t)B * Ho * Wo * Cout, 0.f);
  for (int b = 0; b < B; ++b)
    for (int oh = 0; oh < Ho; ++oh)
      for (int ow = 0; ow < Wo; ++ow)
        for (int n = 0; n < Cout; ++n) {
          double acc = 0;
          for (int kh = 0; kh < k; ++kh)
            for (int kw = 0; kw < k; ++kw) {
              const int ih = oh * s - p + kh, iw = ow * s - p + kw;
              if (ih < 0 || iw < 0 || ih >= H || iw >= W) continue;
              const float* xp = &x[(((size_t)b * H + ih) * W + iw) * Cin];
              const float* wp = &w[(((size_t)n * k + kh) * k + kw) * Cin];
              for (int c = 0; c < Cin; ++c) acc += (double)xp[c] * wp[c];
            }
          y[(((size_t)b * Ho + oh) * Wo + ow) * Cout + n] = (float)acc;
        }
}
static int fp8_check() {
  struct S8 { const char* name; int B, H, W, cin, cout, k, s, p; };
  const S8 shapes[] = {{"3x3 128->128 16x16", 2, 16, 16, 128, 128, 3, 1, 1},
                       {"3x3 64->64 16x16", 2, 16, 16, 64, 64, 3, 1, 1},
                       {"1x1 256->384 8x8", 2, 8, 8, 256, 384, 1, 1, 0},
                       {"4x4s2 64->128 16x16", 2, 16, 16, 64, 128, 4, 2, 1}};
  int fails = 0;
  for (const S8& sh : shapes) {
    const size_t nx = (size_t)sh.B * sh.H * sh.W * sh.cin;
    const int K = sh.k * sh.k * sh.cin, Kp = (K + 127) / 128 * 128;
    std::vector<float> xf(nx), wf((size_t)sh.cout * K);
    uint32_t h = 12345;
    auto rnd = [&]() { h = h * 1664525u + 1013904223u; return ((h >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<bf16> xb(nx);
    for (size_t i = 0; i < nx; ++i) { xb[i] = (bf16)(rnd() * 4.f * (1 + (i % 7))); xf[i] = bf2f(xb[i]); }
    for (auto& v : wf) v = rnd() * 0.2f;
    if (getenv("FP8_ONEHOT")) {         // y[m][n] = (n == m % 128): reveals a permutation
      for (size_t i = 0; i < nx; ++i) { const size_t m = i / sh.cin, c = i % sh.cin; xf[i] = c == m % 128 ? 1.f : 0.f; xb[i] = (bf16)xf[i]; }
      for (size_t i = 0; i < wf.size(); ++i) wf[i] = (i % K) == (i / K) % sh.cin ? 1.f : 0.f;
    }
    std::vector<float> xd, wd;
    std::vector<uint8_t> w8, s8;
    quant_rows(xf, (int)(nx / sh.cin), sh.cin, sh.cin, xd, nullptr, nullptr);   // per pixel, 64-ch blocks
    quant_rows(wf, sh.cout, K, Kp, wd, &w8, &s8);
    int Ho, Wo;
    std::vector<float> yq, yf;
    host_conv(xd, wd, sh.B, sh.H, sh.W, sh.cin, sh.cout, sh.k, sh.s, sh.p, yq, Ho, Wo);
    host_conv(xf, wf, sh.B, sh.H, sh.W, sh.cin, sh.cout, sh.k, sh.s, sh.p, yf, Ho, Wo);
    void *dx, *dy, *dz; uint8_t *dw, *ds;
    CK(hipMalloc(&dx, nx * 2)); CK(hipMalloc(&dy, yq.size() * 2)); CK(hipMalloc(&dz, 256));
    CK(hipMalloc(&dw, w8.size())); CK(hipMalloc(&ds, s8.size()));
    CK(hipMemset(dz, 0, 256));
    CK(hipMemcpy(dx, xb.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, w8.data(), w8.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(ds, s8.data(), s8.size(), hipMemcpyHostToDevice));
    ConvArgs a{};
    a.x1 = dx; a.ld1 = sh.cin; a.C1 = sh.cin; a.Cin = sh.cin; a.Hs = sh.H; a.Ws = sh.W; a.B = sh.B;
    a.Ho = Ho; a.Wo = Wo; a.Cout = sh.cout; a.K = K; a.y = dy; a.ldy = sh.cout; a.zero = dz;
    if (!conv8_ok(a, sh.k, sh.k, sh.s, sh.p)) { printf("fp8 %-22s not eligible\n", sh.name); ++fails; continue; }
    conv8<bf16>(a, sh.k, sh.k, sh.s, sh.p, dw, ds, Kp, 0);
    CK(hipDeviceSynchronize());
    std::vector<bf16> yb(yq.size());
    CK(hipMemcpy(yb.data(), dy, yb.size() * 2, hipMemcpyDeviceToHost));
    double mq = 0, mf = 0, ref = 0;
    int nnan = 0, shown = 0;
    for (size_t i = 0; i < yq.size(); ++i) {
      const float g = bf2f(yb[i]);
      if (!std::isfinite(g)) ++nnan;
      if (shown < 6 && (!std::isfinite(g) || std::fabs(g - yq[i]) > 0.05 * std::fabs(yq[i]) + 0.5)) {
        printf("   m=%zu n=%zu got %g want %g\n", i / sh.cout, i % sh.cout, g, yq[i]);
        ++shown;
      }
      mq = std::max(mq, std::fabs((double)bf2f(yb[i]) - yq[i]));
      mf = std::max(mf, std::fabs((double)bf2f(yb[i]) - yf[i]));
      ref = std::max(ref, std::fabs((double)yf[i]));
    }
    if (getenv("FP8_DUMP")) {
      FILE* f = fopen(getenv("FP8_DUMP"), "a");
      fprintf(f, "%s\n", sh.name);
      for (size_t i = 0; i < yq.size(); ++i)
        if (bf2f(yb[i]) != 0.f) fprintf(f, "%zu %zu %g\n", i / sh.cout, i % sh.cout, bf2f(yb[i]));
      fclose(f);
    }
    if (getenv("FP8_ONEHOT"))
      for (int m = 0; m < 20; ++m) {
        printf("   m=%d nonzero n:", m);
        for (int n = 0; n < std::min(sh.cout, 256); ++n) if (bf2f(yb[(size_t)m * sh.cout + n]) != 0.f) printf(" %d(%g)", n, bf2f(yb[(size_t)m * sh.cout + n]));
        printf("\n");
      }
    if (nnan) printf("   %d non-finite outputs\n", nnan);
    const bool ok = mq / ref < 1e-2 && nnan == 0;
    printf("fp8 %-22s vs quantized-operand ref %.2e (%s), vs exact operands %.2e\n", sh.name, mq / ref,
           ok ? "OK" : "FAIL", mf / ref);
    fails += !ok;
    CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dz)); CK(hipFree(dw)); CK(hipFree(ds));
  }
  return fails;
}

// Input-LayerNorm fold (ConvArgs::lnf_cs, EPI_LNF): LN(x) W^T + b of the SpatialTransformer's
// norm1 -> q|k|v and norm3 -> GEGLU proj against a host fp64 reference of the UNfolded op
// (LayerNorm eps 1e-5 with gain / bias, then the exact-weight GEMM; GEGLU x * gelu(gate) over
// the 16-row interleaved weight layout). x has a per-row offset of several standard deviations
// so the kernel's single-pass moments and its mean * colsum subtraction are exercised.
static int lnf_check(int iters) {
  // (The GEGLU fold tile was deleted in round 4; conv_lnf_ok now rejects ACT_GEGLU.)
  // big: every row's mean is ~3e3 standard deviations off zero (bf16 values there are 16 apart),
  // where one-pass moments E[x^2] - mean^2 lose the variance to fp32 cancellation.
  struct SL { const char* name; int M, C, N, geglu, big; };
  const SL shapes[] = {{"lnf qkv 512->1536", 8192, 512, 1536, 0, 0}, {"lnf qkv 256->768", 8192, 256, 768, 0, 0},
                       {"lnf qkv 512->1536 mean 3e3", 8192, 512, 1536, 0, 1}};
  int fails = 0;
  for (const SL& sh : shapes) {
    const int M = sh.M, C = sh.C, N = sh.N, NO = sh.geglu ? N / 2 : N;
    uint32_t h = 777 + C + N;
    auto rnd = [&]() { h = h * 1664525u + 1013904223u; return ((h >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<bf16> xb((size_t)M * C);
    std::vector<double> xf((size_t)M * C);
    for (int m = 0; m < M; ++m) {
      const float off = sh.big ? 3000.f * (rnd() > 0.f ? 1.f : -1.f) : 6.f * rnd();
      const float sc = sh.big ? 64.f : 0.5f + std::fabs(rnd()) * 2.f;
      for (int c = 0; c < C; ++c) {
        xb[(size_t)m * C + c] = (bf16)(off + sc * rnd());
        xf[(size_t)m * C + c] = bf2f(xb[(size_t)m * C + c]);
      }
    }
    std::vector<float> g(C), be(C), w((size_t)N * C), b(N);
    for (auto& v : g) v = 1.f + 0.5f * rnd();
    for (auto& v : be) v = 0.2f * rnd();
    for (auto& v : w) v = rnd() * 0.1f;
    for (auto& v : b) v = 0.1f * rnd();
    // Folded operands (what engine.cpp Packer::fold_ln stores): w' = bf16(w g), cs = sum w'.
    std::vector<bf16> wf((size_t)N * C);
    std::vector<float> cs(N), bf(N);
    for (int n = 0; n < N; ++n) {
      double c = 0, bb = b[n];
      for (int k = 0; k < C; ++k) {
        wf[(size_t)n * C + k] = (bf16)(w[(size_t)n * C + k] * g[k]);
        c += bf2f(wf[(size_t)n * C + k]);
        bb += (double)w[(size_t)n * C + k] * be[k];
      }
      cs[n] = (float)c;
      bf[n] = (float)bb;
    }
    // Reference (fp64): LN rows, GEMM with the exact weights, bias, GEGLU pairing.
    std::vector<double> ln((size_t)M * C), ref((size_t)M * NO);
    for (int m = 0; m < M; ++m) {
      double mu = 0, var = 0;
      for (int c = 0; c < C; ++c) mu += xf[(size_t)m * C + c];
      mu /= C;
      for (int c = 0; c < C; ++c) { const double d = xf[(size_t)m * C + c] - mu; var += d * d; }
      const double rs = 1.0 / std::sqrt(var / C + 1e-5);
      for (int c = 0; c < C; ++c) ln[(size_t)m * C + c] = (xf[(size_t)m * C + c] - mu) * rs * g[c] + be[c];
    }
    std::vector<double> yr(N);
    for (int m = 0; m < M; ++m) {
      for (int n = 0; n < N; ++n) {
        double acc = b[n];
        const double* lp = &ln[(size_t)m * C];
        const float* wp = &w[(size_t)n * C];
        for (int k = 0; k < C; ++k) acc += lp[k] * wp[k];
        yr[n] = acc;
      }
      for (int o = 0; o < NO; ++o) {
        if (!sh.geglu) { ref[(size_t)m * NO + o] = yr[o]; continue; }
        const int grp = o / 16, s = o % 16;                        // output channel o of group grp
        const double xv = yr[32 * grp + s], gv = yr[32 * grp + 16 + s];
        ref[(size_t)m * NO + o] = xv * 0.5 * gv * (1.0 + std::erf(gv / std::sqrt(2.0)));
      }
    }
    void *dx, *dw, *dy, *dz; float *dcs, *dbf;
    CK(hipMalloc(&dx, xb.size() * 2)); CK(hipMalloc(&dw, wf.size() * 2)); CK(hipMalloc(&dy, (size_t)M * NO * 2));
    CK(hipMalloc(&dz, 256)); CK(hipMalloc(&dcs, N * 4)); CK(hipMalloc(&dbf, N * 4));
    CK(hipMemset(dz, 0, 256));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, wf.data(), wf.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcs, cs.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbf, bf.data(), N * 4, hipMemcpyHostToDevice));
    ConvArgs a{};
    a.x1 = dx; a.ld1 = C; a.C1 = C; a.Cin = C; a.Hs = 32; a.Ws = M / 32 / 8; a.B = 8;
    a.Ho = a.Hs; a.Wo = a.Ws; a.Cout = N; a.K = C; a.w = dw; a.bias = dbf; a.y = dy; a.ldy = NO;
    a.zero = dz; a.act = sh.geglu ? 3 : 0;
    a.lnf_cs = dcs; a.lnf_n = C; a.lnf_eps = 1e-5f;
    if (!conv_lnf_ok(a, 2)) { printf("%-24s not eligible\n", sh.name); ++fails; continue; }
    conv<bf16>(a, 1, 1, 1, 0, 0);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) conv<bf16>(a, 1, 1, 1, 0, 0);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<bf16> yb((size_t)M * NO);
    CK(hipMemcpy(yb.data(), dy, yb.size() * 2, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    int nnan = 0;
    for (size_t i = 0; i < yb.size(); ++i) {
      const double v = bf2f(yb[i]);
      if (!std::isfinite(v)) ++nnan;
      md = std::max(md, std::fabs(v - ref[i]));
      mx = std::max(mx, std::fabs(ref[i]));
    }
    const bool ok = nnan == 0 && md / mx < 1e-2;
    const double us = ms * 1e3 / iters, fl = 2.0 * M * N * C;
    printf("%-24s %8.1f us %7.1f TF/s  check rel %.2e %s\n", sh.name, us, fl / us / 1e6, md / mx, ok ? "OK" : "FAIL");
    fails += !ok;
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dy)); CK(hipFree(dz)); CK(hipFree(dcs)); CK(hipFree(dbf));
  }
  // GroupNorm(32, eps 1e-6) applied in the A path of proj_in (EPI_GNA), stats from the host.
  struct SG { const char* name; int C; };
  const SG gshapes[] = {{"gna proj_in 512->512", 512}, {"gna proj_in 256->256", 256}};
  for (const SG& sh : gshapes) {
    const int B = 8, HW = 1024, M = B * HW, C = sh.C, N = C, G = 32, cpg = C / G;
    uint32_t h = 4242 + C;
    auto rnd = [&]() { h = h * 1664525u + 1013904223u; return ((h >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<bf16> xb((size_t)M * C), wb((size_t)N * C);
    std::vector<float> gm(C), bt(C), bias(N), st((size_t)B * G * 2);
    for (int c = 0; c < C; ++c) { gm[c] = 1.f + 0.5f * rnd(); bt[c] = 0.3f * rnd(); }
    for (int b = 0; b < B; ++b)
      for (int c = 0; c < C; ++c) {
        const float off = 4.f * std::sin(0.37f * (b * C + c)), sc = 1.f + 0.5f * std::cos(0.11f * c);
        for (int p = 0; p < HW; ++p) xb[((size_t)b * HW + p) * C + c] = (bf16)(off + sc * rnd());
      }
    for (auto& v : wb) v = (bf16)(0.1f * rnd());
    for (auto& v : bias) v = 0.1f * rnd();
    std::vector<double> gn((size_t)M * C);
    for (int b = 0; b < B; ++b)
      for (int g = 0; g < G; ++g) {
        double s1 = 0, s2 = 0;
        for (int p = 0; p < HW; ++p)
          for (int c = g * cpg; c < (g + 1) * cpg; ++c) s1 += bf2f(xb[((size_t)b * HW + p) * C + c]);
        const double mu = s1 / (HW * cpg);
        for (int p = 0; p < HW; ++p)
          for (int c = g * cpg; c < (g + 1) * cpg; ++c) { const double d = bf2f(xb[((size_t)b * HW + p) * C + c]) - mu; s2 += d * d; }
        const double rs = 1.0 / std::sqrt(s2 / (HW * cpg) + 1e-6);
        st[((size_t)b * G + g) * 2] = (float)mu;
        st[((size_t)b * G + g) * 2 + 1] = (float)rs;
        for (int p = 0; p < HW; ++p)
          for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            const size_t i = ((size_t)b * HW + p) * C + c;
            gn[i] = (bf2f(xb[i]) - mu) * rs * gm[c] + bt[c];
          }
      }
    std::vector<double> ref((size_t)M * N);
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        double acc = bias[n];
        for (int k = 0; k < C; ++k) acc += gn[(size_t)m * C + k] * bf2f(wb[(size_t)n * C + k]);
        ref[(size_t)m * N + n] = acc;
      }
    void *dx, *dw, *dy, *dz; float *dst, *dg, *db, *dbias;
    CK(hipMalloc(&dx, xb.size() * 2)); CK(hipMalloc(&dw, wb.size() * 2)); CK(hipMalloc(&dy, (size_t)M * N * 2));
    CK(hipMalloc(&dz, 256)); CK(hipMalloc(&dst, st.size() * 4)); CK(hipMalloc(&dg, C * 4)); CK(hipMalloc(&db, C * 4));
    CK(hipMalloc(&dbias, N * 4));
    CK(hipMemset(dz, 0, 256));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, wb.data(), wb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dst, st.data(), st.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, gm.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bt.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbias, bias.data(), N * 4, hipMemcpyHostToDevice));
    ConvArgs a{};
    a.x1 = dx; a.ld1 = C; a.C1 = C; a.Cin = C; a.Hs = 32; a.Ws = 32; a.B = B; a.Ho = 32; a.Wo = 32;
    a.Cout = N; a.K = C; a.w = dw; a.bias = dbias; a.y = dy; a.ldy = N; a.zero = dz;
    a.gna_stats = dst; a.gna_g = dg; a.gna_b = db; a.gna_groups = G;
    if (!conv_gna_ok(a, 2)) { printf("%-24s not eligible\n", sh.name); ++fails; continue; }
    conv<bf16>(a, 1, 1, 1, 0, 0);
    CK(hipDeviceSynchronize());
    {
      // Same GEMM from per-block (sum, sum of squares) over 16-row blocks (ConvArgs::gna_nb):
      // the output must match the (mean, rstd) run to bf16 output rounding.
      const int nbk = HW / 16;
      std::vector<float> ps((size_t)B * G * nbk * 2, 0.f);
      for (int b = 0; b < B; ++b)
        for (int k = 0; k < nbk; ++k)
          for (int p = 16 * k; p < 16 * k + 16; ++p)
            for (int c = 0; c < C; ++c) {
              const double v = bf2f(xb[((size_t)b * HW + p) * C + c]);
              float* q = &ps[(((size_t)b * G + c / cpg) * nbk + k) * 2];
              q[0] += (float)v; q[1] += (float)(v * v);
            }
      float* dps; void* dy2;
      CK(hipMalloc(&dps, ps.size() * 4)); CK(hipMalloc(&dy2, (size_t)M * N * 2));
      CK(hipMemcpy(dps, ps.data(), ps.size() * 4, hipMemcpyHostToDevice));
      ConvArgs a2 = a;
      a2.gna_stats = dps; a2.gna_nb = nbk; a2.gna_eps = 1e-6f; a2.y = dy2;
      conv<bf16>(a2, 1, 1, 1, 0, 0);
      CK(hipDeviceSynchronize());
      std::vector<bf16> y1((size_t)M * N), y2((size_t)M * N);
      CK(hipMemcpy(y1.data(), dy, y1.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(y2.data(), dy2, y2.size() * 2, hipMemcpyDeviceToHost));
      double d = 0, mx2 = 0;
      for (size_t i = 0; i < y1.size(); ++i) { d = std::max(d, (double)std::fabs(bf2f(y1[i]) - bf2f(y2[i]))); mx2 = std::max(mx2, (double)std::fabs(bf2f(y1[i]))); }
      const bool ok2 = d / mx2 < 1e-2;
      printf("%-24s block-sum statistics vs (mean, rstd): rel %.2e  check %s\n", sh.name, d / mx2, ok2 ? "OK" : "FAIL");
      fails += !ok2;
      CK(hipFree(dps)); CK(hipFree(dy2));
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) conv<bf16>(a, 1, 1, 1, 0, 0);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<bf16> yb((size_t)M * N);
    CK(hipMemcpy(yb.data(), dy, yb.size() * 2, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    int nnan = 0;
    for (size_t i = 0; i < yb.size(); ++i) {
      const double v = bf2f(yb[i]);
      if (!std::isfinite(v)) ++nnan;
      md = std::max(md, std::fabs(v - ref[i]));
      mx = std::max(mx, std::fabs(ref[i]));
    }
    const bool ok = nnan == 0 && md / mx < 1e-2;
    const double us = ms * 1e3 / iters, fl = 2.0 * M * N * C;
    printf("%-24s %8.1f us %7.1f TF/s  check rel %.2e %s\n", sh.name, us, fl / us / 1e6, md / mx, ok ? "OK" : "FAIL");
    fails += !ok;
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dy)); CK(hipFree(dz)); CK(hipFree(dst)); CK(hipFree(dg));
    CK(hipFree(db)); CK(hipFree(dbias));
  }
  return fails;
}

// PreNorm LayerNorm with the GroupNorm statistics of its output (norm.hip layernorm_gnstats):
// xn against a host LayerNorm (gain only, eps 1e-5) and the (mean, rstd) table against host
// GroupNorm(32, eps 1e-6) moments of the host LayerNorm output; run twice (the per-image counters
// must come back to zero).
__global__ void fill_rand_h(f16* p, size_t n, uint32_t seed, float scale) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed * 0x9E3779B9u;
  h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12; h *= 0x297a2d39U; h ^= h >> 15;
  p[i] = (f16)(((h >> 8) / 16777216.f - 0.5f) * scale);
}

// LinearAttention block (linattn.hip, fp16) at the UNet's three LA shapes, B = 8: us per call
// of the whole op (la_proj_ctx + la_combine_weff + la_apply; rocprofv3 splits the kernels) and a
// checksum of the output (for comparing builds).
static int la_bench(int iters, float qshift) {
  struct Q { int HW, C; };
  const Q shapes[] = {{256 * 256, 64}, {128 * 128, 128}, {64 * 64, 256}};
  const int B = 8;
  for (const Q& q : shapes) {
    const int C = q.C, HW = q.HW;
    const size_t n = (size_t)B * HW * C;
    f16 *x, *y, *wqkv, *weff; float *gpre, *wout, *bout, *gout, *ws;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&y, n * 2)); CK(hipMalloc(&wqkv, (size_t)3 * 128 * C * 2));
    CK(hipMalloc(&weff, (size_t)B * C * 128 * 2));
    CK(hipMalloc(&gpre, C * 4)); CK(hipMalloc(&wout, (size_t)C * 128 * 4)); CK(hipMalloc(&bout, C * 4)); CK(hipMalloc(&gout, C * 4));
    CK(hipMalloc(&ws, linear_attention_fused_ws_floats(B, HW) * 4));
    fill_rand_h<<<(n + 255) / 256, 256>>>(x, n, 5, 4.f);
    fill_rand_h<<<(3 * 128 * C + 255) / 256, 256>>>(wqkv, 3 * 128 * C, 6, 0.5f);
    fill_rand_f<<<1, 256>>>(gpre, C, 7, 1.f);
    fill_rand_f<<<(C * 128 + 255) / 256, 256>>>(wout, C * 128, 8, 0.2f);
    fill_rand_f<<<1, 256>>>(bout, C, 9, 0.2f);
    fill_rand_f<<<1, 256>>>(gout, C, 10, 1.f);
    auto run = [&]() { linear_attention_fused<f16>(x, wqkv, wout, bout, gout, weff, y, B, HW, C, ws, 0, qshift); };
    run();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) run();
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<f16> h(n);
    CK(hipMemcpy(h.data(), y, n * 2, hipMemcpyDeviceToHost));
    double cs = 0, ca = 0;
    for (size_t i = 0; i < n; ++i) { cs += (double)(float)h[i] * (double)((i % 977) + 1); ca += fabs((float)h[i]); }
    printf("la %3dx%-3d C %3d  %7.1f us/op  checksum %.9e  abs %.9e\n", (int)sqrt((double)HW), (int)sqrt((double)HW), C,
           ms * 1e3 / iters, cs, ca);
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(wqkv)); CK(hipFree(weff)); CK(hipFree(gpre)); CK(hipFree(wout));
    CK(hipFree(bout)); CK(hipFree(gout)); CK(hipFree(ws));
  }
  return 0;
}

static int gns_check() {
  int fails = 0;
  for (int C : {512, 256}) {
    const int B = 8, HW = 1024, M = B * HW, G = 32, cpg = C / G;
    uint32_t h = 99 + C;
    auto rnd = [&]() { h = h * 1664525u + 1013904223u; return ((h >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<bf16> xb((size_t)M * C);
    std::vector<float> g(C);
    for (int c = 0; c < C; ++c) g[c] = 1.f + 0.8f * rnd();
    for (int m = 0; m < M; ++m) {
      const float off = 3.f * rnd();
      for (int c = 0; c < C; ++c) xb[(size_t)m * C + c] = (bf16)(off + (1.f + 0.3f * std::sin(0.05f * c)) * rnd() + 0.2f * std::cos(0.7f * c));
    }
    std::vector<double> ln((size_t)M * C);
    for (int m = 0; m < M; ++m) {
      double mu = 0, var = 0;
      for (int c = 0; c < C; ++c) mu += bf2f(xb[(size_t)m * C + c]);
      mu /= C;
      for (int c = 0; c < C; ++c) { const double d = bf2f(xb[(size_t)m * C + c]) - mu; var += d * d; }
      const double rs = 1.0 / std::sqrt(var / C + 1e-5);
      for (int c = 0; c < C; ++c) ln[(size_t)m * C + c] = (bf2f(xb[(size_t)m * C + c]) - mu) * rs * g[c];
    }
    std::vector<double> st((size_t)B * G * 2);
    for (int b = 0; b < B; ++b)
      for (int gi = 0; gi < G; ++gi) {
        double s1 = 0, s2 = 0;
        for (int p = 0; p < HW; ++p)
          for (int c = gi * cpg; c < (gi + 1) * cpg; ++c) s1 += ln[((size_t)b * HW + p) * C + c];
        const double mu = s1 / (HW * cpg);
        for (int p = 0; p < HW; ++p)
          for (int c = gi * cpg; c < (gi + 1) * cpg; ++c) { const double d = ln[((size_t)b * HW + p) * C + c] - mu; s2 += d * d; }
        st[((size_t)b * G + gi) * 2] = mu;
        st[((size_t)b * G + gi) * 2 + 1] = 1.0 / std::sqrt(s2 / (HW * cpg) + 1e-6);
      }
    void *dx, *dy; float *dg, *dpart;
    const size_t wsf = layernorm_gnstats_ws_floats(B, HW, G);
    CK(hipMalloc(&dx, xb.size() * 2)); CK(hipMalloc(&dy, xb.size() * 2)); CK(hipMalloc(&dg, C * 4));
    CK(hipMalloc(&dpart, wsf * 4));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, g.data(), C * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(dpart, 0xff, wsf * 4));
      const int nb = layernorm_gnstats<bf16>(dx, C, dy, C, dg, nullptr, M, C, 1e-5f, HW, G, dpart, true, 0);
      if (nb <= 0) { printf("gns C=%d not eligible\n", C); ++fails; break; }
      CK(hipDeviceSynchronize());
      std::vector<bf16> yb(xb.size());
      std::vector<float> pt((size_t)B * G * nb * 2);
      CK(hipMemcpy(yb.data(), dy, yb.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(pt.data(), dpart, pt.size() * 4, hipMemcpyDeviceToHost));
      double ey = 0, my = 0, em = 0, er = 0;
      for (size_t i = 0; i < yb.size(); ++i) { ey = std::max(ey, std::fabs(bf2f(yb[i]) - ln[i])); my = std::max(my, std::fabs(ln[i])); }
      for (int i = 0; i < B * G; ++i) {        // merge the block sums as proj_in's table fill does
        double s1 = 0, s2 = 0;
        for (int k = 0; k < nb; ++k) { s1 += pt[((size_t)i * nb + k) * 2]; s2 += pt[((size_t)i * nb + k) * 2 + 1]; }
        const double n = (double)HW * cpg, mu = s1 / n, rs = 1.0 / std::sqrt(std::max(s2 / n - mu * mu, 0.0) + 1e-6);
        em = std::max(em, std::fabs(mu - st[2 * i]));
        er = std::max(er, std::fabs(rs - st[2 * i + 1]) / st[2 * i + 1]);
      }
      const bool ok = ey / my < 1e-2 && em < 1e-4 && er < 1e-4;
      printf("gns C=%d rep %d: %d blocks/image, xn rel %.2e, mean abs %.2e, rstd rel %.2e  check %s\n", C, rep, nb,
             ey / my, em, er, ok ? "OK" : "FAIL");
      fails += !ok;
    }
    CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dg)); CK(hipFree(dpart));
  }
  return fails;
}

// ---- fp8 ResBlock pair (conv3q.hip): block1 with an e4m3 output (v5 64 -> 64, or the fused
// res_conv v4 tiles on a 64 | 64 concat), then block2 on the e4m3 tensor.
//  producer: the dequantized e4m3 output against the same conv's 16-bit output (e4m3 rounding:
//    |d - y| <= 2^-4 |y| + 2^(e - 9) per value, e the block exponent, plus the 16-bit rounding),
//    every block exponent the smallest (+-1 at a rounding boundary) with max / 2^e <= 448, and
//    the fused res_conv output identical to the 16-bit run's;
//  consumer: against a host fp64 conv of the dequantized input and weights with the same
//    epilogue (bias, SiLU, + res1), max-rel < 1e-2 (bf16 output rounding);
//  then times the pair against the 16-bit pair at B = 8, 256^2 (the bench level) and 128^2.
static void q8_weights(const std::vector<float>& w, std::vector<uint8_t>& w8, std::vector<uint8_t>& s8,
                       std::vector<float>& deq) {
  // w: [64][3][3][64] -> e4m3 [64][9][64] + E8M0 [64][9][2] (engine.cpp Packer::make_q8c3)
  w8.assign(64 * 576, 0); s8.assign(64 * 18, 127); deq.assign(64 * 576, 0.f);
  for (int n = 0; n < 64; ++n)
    for (int t = 0; t < 9; ++t)
      for (int h = 0; h < 2; ++h) {
        const size_t o = (size_t)n * 576 + t * 64 + 32 * h;
        float mx = 0.f;
        for (int c = 0; c < 32; ++c) mx = std::max(mx, std::fabs(w[o + c]));
        int e = mx > 0.f ? (int)std::ceil(std::log2((double)mx / 448.0)) : 0;
        e = std::min(126, std::max(-126, e));
        s8[(size_t)n * 18 + t * 2 + h] = (uint8_t)(127 + e);
        for (int c = 0; c < 32; ++c) {
          w8[o + c] = f2e4m3(std::ldexp(w[o + c], -e));
          deq[o + c] = std::ldexp(e4m3f(w8[o + c]), e);
        }
      }
}
static int q8_check(int iters) {
  int fails = 0;
  struct Q { const char* name; int B, H, W, cin1; bool check; };
  const Q shapes[] = {{"q8 check 64->64 16x128", 2, 16, 128, 64, true},
                      {"q8 check 64|64->64 +1x1 8x256", 1, 8, 256, 128, true},
                      {"q8 256x256 B8 64->64", 8, 256, 256, 64, false},
                      {"q8 256x256 B8 64|64->64 +1x1", 8, 256, 256, 128, false},
                      {"q8 128x128 B8 64->64", 8, 128, 128, 64, false}};
  for (const Q& sh : shapes) {
    const int B = sh.B, H = sh.H, W = sh.W, C1 = sh.cin1, M = B * H * W;
    const bool res_in = C1 == 128;
    uint32_t hs = 777 + C1 + W;
    auto rnd = [&]() { hs = hs * 1664525u + 1013904223u; return ((hs >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<bf16> xb((size_t)M * C1), rb((size_t)M * 64), w1b((size_t)64 * 9 * C1), w2rb((size_t)64 * C1);
    for (size_t i = 0; i < xb.size(); ++i) xb[i] = (bf16)(2.f * rnd() * (1 + (i / C1) % 5));
    for (auto& v : rb) v = (bf16)rnd();
    for (auto& v : w1b) v = (bf16)(0.1f * rnd());
    for (auto& v : w2rb) v = (bf16)(0.1f * rnd());
    std::vector<float> ss((size_t)B * 128), bias2(64), w2f((size_t)64 * 576);
    for (auto& v : ss) v = 0.5f * rnd();
    for (auto& v : bias2) v = 0.2f * rnd();
    for (auto& v : w2f) v = 0.08f * rnd();
    std::vector<uint8_t> q8w, q8s;
    std::vector<float> w2d;
    q8_weights(w2f, q8w, q8s, w2d);
    std::vector<bf16> w2b(w2f.size());
    for (size_t i = 0; i < w2f.size(); ++i) w2b[i] = (bf16)w2f[i];
    void *dx, *dr, *dw1, *dw2r, *dh16, *dy2a, *dy2b, *dz, *dout, *dout16, *dw2b;
    float *dss, *db2; uint8_t *dh8, *dhs, *dq8w, *dq8s;
    CK(hipMalloc(&dx, xb.size() * 2)); CK(hipMalloc(&dr, rb.size() * 2)); CK(hipMalloc(&dw1, w1b.size() * 2));
    CK(hipMalloc(&dw2r, w2rb.size() * 2)); CK(hipMalloc(&dh16, (size_t)M * 128)); CK(hipMalloc(&dy2a, (size_t)M * 128));
    CK(hipMalloc(&dy2b, (size_t)M * 128)); CK(hipMalloc(&dz, 256)); CK(hipMalloc(&dout, (size_t)M * 128));
    CK(hipMalloc(&dout16, (size_t)M * 128)); CK(hipMalloc(&dw2b, w2b.size() * 2));
    CK(hipMalloc(&dss, ss.size() * 4)); CK(hipMalloc(&db2, 256)); CK(hipMalloc(&dh8, (size_t)M * 64));
    CK(hipMalloc(&dhs, (size_t)M * 2)); CK(hipMalloc(&dq8w, q8w.size())); CK(hipMalloc(&dq8s, q8s.size()));
    CK(hipMemset(dz, 0, 256));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, rb.data(), rb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw1, w1b.data(), w1b.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw2r, w2rb.data(), w2rb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw2b, w2b.data(), w2b.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dss, ss.data(), ss.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db2, bias2.data(), 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(dq8w, q8w.data(), q8w.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dq8s, q8s.data(), q8s.size(), hipMemcpyHostToDevice));
    // block1: x (64, or 64 | 64 as x1 | x2) -> h, scale/shift + SiLU (+ the fused 1x1 res_conv)
    ConvArgs a1{};
    a1.x1 = dx; a1.ld1 = C1; a1.C1 = C1; a1.Cin = C1;
    if (res_in) { a1.x2 = (const bf16*)dx + 64; a1.ld2 = C1; a1.C1 = 64; }
    a1.Hs = H; a1.Ws = W; a1.B = B; a1.Ho = H; a1.Wo = W; a1.Cout = 64; a1.K = 9 * C1; a1.w = dw1;
    a1.ss = dss; a1.ss_ld = 128; a1.act = 1; a1.zero = dz; a1.y = dh16; a1.ldy = 64;
    if (res_in) { a1.w2 = dw2r; a1.y2 = dy2a; a1.ldy2 = 64; }
    ConvArgs a1q = a1;
    a1q.y = dh8; a1q.ys8 = dhs;
    if (res_in) a1q.y2 = dy2b;
    if (!conv_q8out_ok(a1q)) { printf("%-32s producer not eligible\n", sh.name); ++fails; continue; }
    // block2: h -> out, SiLU, + res (the 16-bit pair reads h16 with the bf16-rounded weights)
    ConvArgs a2{};
    a2.x1 = dh16; a2.ld1 = 64; a2.C1 = 64; a2.Cin = 64; a2.Hs = H; a2.Ws = W; a2.B = B; a2.Ho = H; a2.Wo = W;
    a2.Cout = 64; a2.K = 576; a2.w = dw2b; a2.bias = db2; a2.act = 1; a2.zero = dz; a2.res1 = dr; a2.ldr1 = 64;
    a2.y = dout16; a2.ldy = 64;
    ConvArgs a2q = a2;
    a2q.x1 = dh8; a2q.xs8 = dhs; a2q.y = dout; a2q.w = nullptr;
    if (!conv3q_ok(a2q)) { printf("%-32s consumer not eligible\n", sh.name); ++fails; continue; }
    conv<bf16>(a1, 3, 3, 1, 1, 0);
    conv<bf16>(a1q, 3, 3, 1, 1, 0);
    conv3q<bf16>(a2q, dq8w, dq8s, 0);
    conv<bf16>(a2, 3, 3, 1, 1, 0);
    CK(hipDeviceSynchronize());
    if (sh.check) {
      std::vector<bf16> h16((size_t)M * 64), y2a, y2b, o((size_t)M * 64);
      std::vector<uint8_t> h8((size_t)M * 64), e8((size_t)M * 2);
      CK(hipMemcpy(h16.data(), dh16, h16.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h8.data(), dh8, h8.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(e8.data(), dhs, e8.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(o.data(), dout, o.size() * 2, hipMemcpyDeviceToHost));
      int bad_v = 0, bad_e = 0;
      std::vector<float> hd((size_t)M * 64);
      for (int m = 0; m < M; ++m)
        for (int hf = 0; hf < 2; ++hf) {
          const int e = (int)e8[(size_t)m * 2 + hf] - 127;
          float mx = 0.f, mq = 0.f;
          for (int c = 32 * hf; c < 32 * hf + 32; ++c) {
            const size_t i = (size_t)m * 64 + c;
            const float y = bf2f(h16[i]), d = std::ldexp(e4m3f(h8[i]), e);
            hd[i] = d;
            mx = std::max(mx, std::fabs(y));
            mq = std::max(mq, std::fabs(e4m3f(h8[i])));
            if (!(std::fabs(d - y) <= 0.0703f * std::fabs(y) + std::ldexp(1.f, e - 8))) {
              if (bad_v < 4) printf("   h m=%d c=%d got %g want %g (e %d)\n", m, c, d, y, e);
              ++bad_v;
            }
          }
          const int eh = mx > 0.f ? (int)std::ceil(std::log2(mx / 440.0)) : -126;
          if (mq > 448.f || std::abs(e - std::max(-126, eh)) > 1) {
            if (bad_e < 4) printf("   exponent m=%d half %d: %d (host %d, max code %g)\n", m, hf, e, eh, mq);
            ++bad_e;
          }
        }
      if (res_in) {
        y2a.resize((size_t)M * 64); y2b.resize((size_t)M * 64);
        CK(hipMemcpy(y2a.data(), dy2a, (size_t)M * 128, hipMemcpyDeviceToHost));
        CK(hipMemcpy(y2b.data(), dy2b, (size_t)M * 128, hipMemcpyDeviceToHost));
        if (memcmp(y2a.data(), y2b.data(), (size_t)M * 128)) { printf("   fused res_conv output differs\n"); ++bad_v; }
      }
      double md = 0, mref = 0;
      int shown = 0;
      for (int b = 0; b < B; ++b)
        for (int oh = 0; oh < H; ++oh)
          for (int ow = 0; ow < W; ++ow)
            for (int n = 0; n < 64; ++n) {
              double acc = 0;
              for (int kh = 0; kh < 3; ++kh)
                for (int kw = 0; kw < 3; ++kw) {
                  const int ih = oh + kh - 1, iw = ow + kw - 1;
                  if (ih < 0 || iw < 0 || ih >= H || iw >= W) continue;
                  const float* xp = &hd[(((size_t)b * H + ih) * W + iw) * 64];
                  const float* wp = &w2d[(size_t)n * 576 + (kh * 3 + kw) * 64];
                  for (int c = 0; c < 64; ++c) acc += (double)xp[c] * wp[c];
                }
              acc += bias2[n];
              acc = acc / (1.0 + std::exp(-acc));
              const size_t i = (((size_t)b * H + oh) * W + ow) * 64 + n;
              acc += bf2f(rb[i]);
              const double g = bf2f(o[i]);
              if (shown < 4 && !(std::fabs(g - acc) <= 1e-2 * std::max(1.0, std::fabs(acc)))) {
                printf("   out b=%d oh=%d ow=%d n=%d got %g want %g\n", b, oh, ow, n, g, acc);
                ++shown;
              }
              md = std::max(md, std::fabs(g - acc));
              mref = std::max(mref, std::fabs(acc));
            }
      const bool ok = bad_v == 0 && bad_e == 0 && md / mref < 1e-2;
      printf("%-32s producer: %d bad values, %d bad exponents; consumer rel %.2e  check %s\n", sh.name, bad_v, bad_e,
             md / mref, ok ? "OK" : "FAIL");
      fails += !ok;
    } else {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      auto tm = [&](auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) fn();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3 / iters;
      };
      double t1 = tm([&] { conv<bf16>(a1, 3, 3, 1, 1, 0); });
      double t1q = tm([&] { conv<bf16>(a1q, 3, 3, 1, 1, 0); });
      // (second, interleaved pass: the chip's clock drifts between the first launches)
      t1 = std::min(t1, tm([&] { conv<bf16>(a1, 3, 3, 1, 1, 0); }));
      t1q = std::min(t1q, tm([&] { conv<bf16>(a1q, 3, 3, 1, 1, 0); }));
      const double t2 = tm([&] { conv<bf16>(a2, 3, 3, 1, 1, 0); });
      const double t2q = tm([&] { conv3q<bf16>(a2q, dq8w, dq8s, 0); });
      const double fl2 = 2.0 * M * 64 * 576;
      printf("%-32s block1 16-bit %6.1f us, e4m3 out %6.1f us | block2 16-bit %6.1f us (%5.0f TF/s), e4m3 %6.1f us "
             "(%5.0f TF/s) | pair %6.1f -> %6.1f us\n", sh.name, t1, t1q, t2, fl2 / t2 / 1e6, t2q, fl2 / t2q / 1e6,
             t1 + t2, t1q + t2q);
      CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    }
    for (void* p : {dx, dr, dw1, dw2r, dh16, dy2a, dy2b, dz, dout, dout16, dw2b}) CK(hipFree(p));
    for (void* p : {(void*)dss, (void*)db2, (void*)dh8, (void*)dhs, (void*)dq8w, (void*)dq8s}) CK(hipFree(p));
  }
  return fails;
}

// ---- row-phase upsample conv (ConvArgs::uph): the UNet's Upsample convs (nearest 2x, then
// 3x3) as two kernel rows per output-row parity with summed weights, against the plain up conv
// with the same fp32 weights (each rounded to bf16: the folded rows round once, so the bound
// is the bf16 rounding, max-rel < 1e-2), then both timed at B = 8.
template <typename E> static int uph_check(int iters, const char* tn) {
  struct U { const char* name; int B, Hs, Ws, cin, cout; };
  const U shapes[] = {{"uph 128^2->256^2 128->64", 8, 128, 128, 128, 64},
                      {"uph 64^2->128^2 256->128", 8, 64, 64, 256, 128},
                      {"uph 32^2->64^2 512->256", 8, 32, 32, 512, 256}};
  int fails = 0;
  for (const U& sh : shapes) {
    const int Ho = 2 * sh.Hs, Wo = 2 * sh.Ws, M = sh.B * Ho * Wo, C = sh.cin, N = sh.cout;
    uint32_t hs = 4242 + C;
    auto rnd = [&]() { hs = hs * 1664525u + 1013904223u; return ((hs >> 8) & 0xffff) / 65535.f - 0.5f; };
    std::vector<E> xb((size_t)sh.B * sh.Hs * sh.Ws * C), wb((size_t)N * 9 * C), pb((size_t)N * 12 * C),
        qb((size_t)N * 16 * C);
    std::vector<float> wf((size_t)N * 9 * C), bias(N);
    for (auto& v : xb) v = (E)(2.f * rnd());
    for (auto& v : wf) v = 0.05f * rnd();
    for (auto& v : bias) v = 0.1f * rnd();
    for (size_t i = 0; i < wf.size(); ++i) wb[i] = (E)wf[i];
    const size_t R = (size_t)3 * C;
    for (int o = 0; o < N; ++o)
      for (size_t k = 0; k < R; ++k) {
        const float* w = &wf[(size_t)o * 3 * R];
        E* d = &pb[(size_t)o * 4 * R];
        d[k] = (E)w[k]; d[R + k] = (E)(w[R + k] + w[2 * R + k]);
        d[2 * R + k] = (E)(w[k] + w[R + k]); d[3 * R + k] = (E)w[2 * R + k];
      }
    {
      static const int lo[4] = {0, 1, 0, 2}, hi[4] = {0, 2, 1, 2};
      for (int o = 0; o < N; ++o)
        for (int rs = 0; rs < 4; ++rs)
          for (int cs = 0; cs < 4; ++cs)
            for (int c = 0; c < C; ++c) {
              float v = 0.f;
              for (int kh = lo[rs]; kh <= hi[rs]; ++kh)
                for (int kw = lo[cs]; kw <= hi[cs]; ++kw) v += wf[(((size_t)o * 3 + kh) * 3 + kw) * C + c];
              qb[(((size_t)o * 4 + rs) * 4 + cs) * C + c] = (E)v;
            }
    }
    void *dx, *dw, *dp, *dq, *dz, *dy0, *dy1, *dy2; float* db;
    CK(hipMalloc(&dq, qb.size() * 2)); CK(hipMalloc(&dy2, (size_t)M * N * 2));
    CK(hipMemcpy(dq, qb.data(), qb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMalloc(&dx, xb.size() * 2)); CK(hipMalloc(&dw, wb.size() * 2)); CK(hipMalloc(&dp, pb.size() * 2));
    CK(hipMalloc(&dz, 256)); CK(hipMalloc(&dy0, (size_t)M * N * 2)); CK(hipMalloc(&dy1, (size_t)M * N * 2));
    CK(hipMalloc(&db, N * 4));
    CK(hipMemset(dz, 0, 256));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, wb.data(), wb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp, pb.data(), pb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
    ConvArgs a{};
    a.x1 = dx; a.ld1 = C; a.C1 = C; a.Cin = C; a.Hs = sh.Hs; a.Ws = sh.Ws; a.up = 1; a.B = sh.B; a.Ho = Ho;
    a.Wo = Wo; a.Cout = N; a.K = 9 * C; a.w = dw; a.bias = db; a.zero = dz; a.y = dy0; a.ldy = N;
    ConvArgs u = a;
    u.w = dp; u.K = 12 * C; u.uph = 1; u.y = dy1;
    ConvArgs u2 = a;
    u2.w = dq; u2.K = 16 * C; u2.uph = 2; u2.y = dy2;
    const bool col = conv_uph_ok(u2);
    if (!conv_uph_ok(u)) { printf("%s %-28s not eligible\n", tn, sh.name); ++fails; continue; }
    conv<E>(a, 3, 3, 1, 1, 0);
    conv<E>(u, 3, 3, 1, 1, 0);
    if (col) conv<E>(u2, 3, 3, 1, 1, 0);
    CK(hipDeviceSynchronize());
    std::vector<E> y0((size_t)M * N), y1((size_t)M * N), y2((size_t)M * N);
    CK(hipMemcpy(y0.data(), dy0, y0.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y1.data(), dy1, y1.size() * 2, hipMemcpyDeviceToHost));
    if (col) CK(hipMemcpy(y2.data(), dy2, y2.size() * 2, hipMemcpyDeviceToHost));
    double md = 0, mx = 0, md2 = 0;
    for (size_t i = 0; i < y0.size(); ++i) {
      md = std::max(md, std::fabs((double)bf2f(y1[i]) - bf2f(y0[i])));
      if (col) md2 = std::max(md2, std::fabs((double)bf2f(y2[i]) - bf2f(y0[i])));
      mx = std::max(mx, std::fabs((double)bf2f(y0[i])));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto tm = [&](const ConvArgs& c) {
      for (int i = 0; i < 3; ++i) conv<E>(c, 3, 3, 1, 1, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) conv<E>(c, 3, 3, 1, 1, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1e3 / iters;
    };
    double t0 = tm(a), t1 = tm(u), t2 = col ? tm(u2) : 0.0;
    t0 = std::min(t0, tm(a));
    t1 = std::min(t1, tm(u));
    if (col) t2 = std::min(t2, tm(u2));
    const bool ok = md / mx < 1e-2 && md2 / mx < 1e-2;
    printf("%s %-28s plain %6.1f us, row-phase %6.1f us, row+column %6.1f us  check rel %.2e / %.2e %s\n", tn, sh.name, t0,
           t1, t2, md / mx, md2 / mx, ok ? "OK" : "FAIL");
    fails += !ok;
    for (void* p : {dx, dw, dp, dq, dz, dy0, dy1, dy2, (void*)db}) CK(hipFree(p));
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  }
  return fails;
}


// ---- conv3r (conv3r.hip) check: two-source inputs (torch.cat of x1 | x2 with different pitches),
// the fused 1x1 res_conv output y2, residual / scale-shift / SiLU epilogues, against a host fp64
// recomputation at sampled outputs; timed against the kernel the dispatcher takes without it.
static int c3r_check(int iters) {
  struct Q { const char* name; int B, H, W, c1, c2, ld2, act, ss, res, fuse; };
  const Q shapes[] = {
    {"c3r 64->64 ss+silu", 2, 256, 256, 64, 0, 0, 1, 1, 0, 0},
    {"c3r 64->64 silu+res", 2, 256, 256, 64, 0, 0, 1, 0, 1, 0},
    {"c3r 64->64 plain 256x512", 1, 256, 512, 64, 0, 0, 0, 0, 0, 0},
    {"c3r 64|64->64 ss+silu +1x1", 2, 256, 256, 64, 64, 96, 1, 1, 0, 1},
    {"c3r 128->64 silu +1x1 256x512", 1, 256, 512, 128, 0, 0, 1, 0, 0, 1},
    {"c3r 128->64 ss+silu", 2, 256, 256, 128, 0, 0, 1, 1, 0, 0},
    {"c3r 64|64->64 ss+silu +1x1 B8", 8, 256, 256, 64, 64, 64, 1, 1, 0, 1},
  };
  int bad = 0;
  for (const Q& q : shapes) {
    const int cin = q.c1 + q.c2, ld1 = q.c1, ld2 = q.c2 ? q.ld2 : 0;
    const size_t npx = (size_t)q.B * q.H * q.W;
    const size_t nw = (size_t)64 * 9 * cin, nw2 = (size_t)64 * cin;
    bf16 *x1, *x2 = nullptr, *w, *w2, *y, *y2, *res;
    float *ss, *bias;
    CK(hipMalloc(&x1, npx * ld1 * 2)); if (q.c2) CK(hipMalloc(&x2, npx * ld2 * 2));
    CK(hipMalloc(&w, nw * 2)); CK(hipMalloc(&w2, nw2 * 2)); CK(hipMalloc(&y, npx * 64 * 2));
    CK(hipMalloc(&y2, npx * 64 * 2)); CK(hipMalloc(&res, npx * 64 * 2));
    CK(hipMalloc(&ss, q.B * 128 * 4)); CK(hipMalloc(&bias, 64 * 4));
    fill_rand<<<(npx * ld1 + 255) / 256, 256>>>(x1, npx * ld1, 11, 2.f);
    if (q.c2) fill_rand<<<(npx * ld2 + 255) / 256, 256>>>(x2, npx * ld2, 12, 2.f);
    fill_rand<<<(nw + 255) / 256, 256>>>(w, nw, 13, 0.1f);
    fill_rand<<<(nw2 + 255) / 256, 256>>>(w2, nw2, 14, 0.2f);
    fill_rand<<<(npx * 64 + 255) / 256, 256>>>(res, npx * 64, 15, 2.f);
    fill_rand_f<<<1, 256>>>(ss, q.B * 128, 16, 1.f);
    fill_rand_f<<<1, 64>>>(bias, 64, 17, 1.f);
    void* zero; CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
    ConvArgs a{};
    a.x1 = x1; a.ld1 = ld1; a.C1 = q.c1; a.x2 = x2; a.ld2 = ld2; a.Cin = cin; a.Hs = q.H; a.Ws = q.W;
    a.B = q.B; a.Ho = q.H; a.Wo = q.W; a.Cout = 64; a.K = 9 * cin; a.w = w; a.y = y; a.ldy = 64;
    a.act = q.act; a.bias = bias; a.zero = zero;
    if (q.ss) { a.ss = ss; a.ss_ld = 128; }
    if (q.res) { a.res1 = res; a.ldr1 = 64; }
    if (q.fuse) { a.w2 = w2; a.y2 = y2; a.ldy2 = 64; }
    double t[2] = {0, 0};
    std::vector<bf16> hy(npx * 64), hy2(q.fuse ? npx * 64 : 0);
    for (int arm = 1; arm >= 0; --arm) {                     // 1: conv3r, 0: without it
      dac_conv3r_enable(arm);
      dac_conv3_force(-1);
      if (q.fuse && !conv_res_fusable(a)) { printf("%-32s arm %d: no fused kernel\n", q.name, arm); continue; }
      conv<bf16>(a, 3, 3, 1, 1, 0);
      CK(hipDeviceSynchronize());
      if (arm == 1) {
        printf("%-32s variant %d", q.name, conv_variant(a, 3, 2));
        CK(hipMemcpy(hy.data(), y, npx * 64 * 2, hipMemcpyDeviceToHost));
        if (q.fuse) CK(hipMemcpy(hy2.data(), y2, npx * 64 * 2, hipMemcpyDeviceToHost));
      }
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) conv<bf16>(a, 3, 3, 1, 1, 0);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      t[arm] = ms * 1e3 / iters;
    }
    dac_conv3r_enable(1);
    // Host fp64 reference at sampled outputs.
    std::vector<bf16> hx1(npx * ld1), hx2(q.c2 ? npx * ld2 : 0), hw(nw), hw2(nw2), hr(npx * 64);
    std::vector<float> hss(q.B * 128), hb(64);
    CK(hipMemcpy(hx1.data(), x1, hx1.size() * 2, hipMemcpyDeviceToHost));
    if (q.c2) CK(hipMemcpy(hx2.data(), x2, hx2.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hw.data(), w, nw * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hw2.data(), w2, nw2 * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), res, hr.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hss.data(), ss, hss.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), bias, 256, hipMemcpyDeviceToHost));
    auto xin = [&](size_t pix, int c) -> double {
      return c < q.c1 ? bf2f(hx1[pix * ld1 + c]) : bf2f(hx2[pix * ld2 + c - q.c1]);
    };
    double d1 = 0, m1 = 0, d2 = 0, m2 = 0;
    uint32_t st = 777u;
    for (int k = 0; k < 4096; ++k) {
      st = st * 1664525u + 1013904223u;
      const size_t i = ((size_t)st * 2654435761u) % (npx * 64);
      const int n = (int)(i % 64);
      const size_t m = i / 64;
      const int b = (int)(m / ((size_t)q.H * q.W)), rr = (int)(m % ((size_t)q.H * q.W)), oh = rr / q.W, ow = rr % q.W;
      double acc = 0, acc2 = 0;
      for (int ky = 0; ky < 3; ++ky)
        for (int kx = 0; kx < 3; ++kx) {
          const int ih = oh - 1 + ky, iw = ow - 1 + kx;
          if (ih < 0 || iw < 0 || ih >= q.H || iw >= q.W) continue;
          const size_t pix = ((size_t)b * q.H + ih) * q.W + iw;
          for (int c = 0; c < cin; ++c) acc += xin(pix, c) * bf2f(hw[((size_t)n * 9 + ky * 3 + kx) * cin + c]);
        }
      for (int c = 0; c < cin; ++c) acc2 += xin(m, c) * bf2f(hw2[(size_t)n * cin + c]);
      acc += hb[n];
      if (q.ss) acc = acc * (hss[b * 128 + n] + 1.0) + hss[b * 128 + 64 + n];
      if (q.act == 1) acc = acc / (1.0 + std::exp(-acc));
      if (q.res) acc += bf2f(hr[m * 64 + n]);
      d1 = fmax(d1, fabs((double)bf2f(hy[m * 64 + n]) - acc)); m1 = fmax(m1, fabs(acc));
      if (q.fuse) { d2 = fmax(d2, fabs((double)bf2f(hy2[m * 64 + n]) - acc2)); m2 = fmax(m2, fabs(acc2)); }
    }
    const bool ok = d1 / m1 < 1e-2 && (!q.fuse || d2 / m2 < 1e-2);
    bad += !ok;
    printf("  conv3r %7.1f us, without %7.1f us  host rel %.2e", t[1], t[0], d1 / m1);
    if (q.fuse) printf(" y2 rel %.2e", d2 / m2);
    printf("  check %s\n", ok ? "OK" : "FAIL");
    hipFree(x1); if (x2) hipFree(x2); hipFree(w); hipFree(w2); hipFree(y); hipFree(y2); hipFree(res);
    hipFree(ss); hipFree(bias); hipFree(zero);
  }
  return bad ? 1 : 0;
}

// ---- fused ResBlock (rbfuse.hip) check: the single launch must reproduce the two-launch pair
// (block1 3x3 + scale/shift + SiLU [+ fused 1x1 res_conv], block2 3x3 + SiLU + residual) bit for
// bit — both are the same ordered MFMA sums and epilogue arithmetic — and is timed against it.
template <typename E> __global__ void fill_rand_t(E* p, size_t n, uint32_t seed, float scale) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed * 0x9e3779b9u;
  h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
  p[i] = (E)(((h & 0xffff) / 65535.f - 0.5f) * scale);
}

template <typename E> static int rbf_check(int iters, const char* tn) {
  struct Q { const char* name; int B, H, W, c1, c2, ld2; };
  const Q shapes[] = {
    {"rbf 64->64 x1 256^2", 1, 256, 256, 64, 0, 0},
    {"rbf 64|64->64 x1 256^2", 1, 256, 256, 64, 64, 64},
    {"rbf 64->64 x2 256^2", 2, 256, 256, 64, 0, 0},
    {"rbf 128->64 256x512", 1, 256, 512, 128, 0, 0},
    {"rbf 64|64->64 256^2 ld2 96", 2, 256, 256, 64, 64, 96},
    {"rbf 64->64 B4 256^2", 4, 256, 256, 64, 0, 0},
    {"rbf 64|64->64 B4 256^2", 4, 256, 256, 64, 64, 64},
    {"rbf 64->64 B8 256^2", 8, 256, 256, 64, 0, 0},
    {"rbf 64|64->64 B8 256^2", 8, 256, 256, 64, 64, 64},
  };
  int bad = 0;
  for (const Q& q : shapes) {
    const int cin = q.c1 + q.c2, ld1 = q.c1, ld2 = q.c2 ? q.ld2 : 0;
    const bool res = cin == 128;
    const size_t npx = (size_t)q.B * q.H * q.W;
    E *x1, *x2 = nullptr, *w1, *w2, *wr, *h, *y2, *yu, *yf;
    float* ss;
    CK(hipMalloc(&x1, npx * ld1 * 2)); if (q.c2) CK(hipMalloc(&x2, npx * ld2 * 2));
    CK(hipMalloc(&w1, (size_t)64 * 9 * cin * 2)); CK(hipMalloc(&w2, (size_t)64 * 576 * 2)); CK(hipMalloc(&wr, (size_t)64 * cin * 2));
    CK(hipMalloc(&h, npx * 128)); CK(hipMalloc(&y2, npx * 128)); CK(hipMalloc(&yu, npx * 128)); CK(hipMalloc(&yf, npx * 128));
    CK(hipMalloc(&ss, q.B * 128 * 4));
    fill_rand_t<E><<<(npx * ld1 + 255) / 256, 256>>>(x1, npx * ld1, 21, 2.f);
    if (q.c2) fill_rand_t<E><<<(npx * ld2 + 255) / 256, 256>>>(x2, npx * ld2, 22, 2.f);
    fill_rand_t<E><<<(64 * 9 * cin + 255) / 256, 256>>>(w1, (size_t)64 * 9 * cin, 23, 0.1f);
    fill_rand_t<E><<<(64 * 576 + 255) / 256, 256>>>(w2, (size_t)64 * 576, 24, 0.1f);
    fill_rand_t<E><<<(64 * cin + 255) / 256, 256>>>(wr, (size_t)64 * cin, 25, 0.2f);
    fill_rand_f<<<(q.B * 128 + 255) / 256, 256>>>(ss, q.B * 128, 26, 1.f);
    void* zero; CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
    ConvArgs a1{};
    a1.x1 = x1; a1.ld1 = ld1; a1.C1 = q.c1; a1.x2 = x2; a1.ld2 = ld2; a1.Cin = cin; a1.Hs = q.H; a1.Ws = q.W;
    a1.B = q.B; a1.Ho = q.H; a1.Wo = q.W; a1.Cout = 64; a1.K = 9 * cin; a1.w = w1; a1.y = h; a1.ldy = 64;
    a1.act = 1; a1.zero = zero; a1.ss = ss; a1.ss_ld = 128;
    if (res) { a1.w2 = wr; a1.y2 = y2; a1.ldy2 = 64; }
    ConvArgs a2{};
    a2.x1 = h; a2.ld1 = 64; a2.C1 = 64; a2.Cin = 64; a2.Hs = q.H; a2.Ws = q.W; a2.B = q.B; a2.Ho = q.H; a2.Wo = q.W;
    a2.Cout = 64; a2.K = 576; a2.w = w2; a2.y = yu; a2.ldy = 64; a2.act = 1; a2.zero = zero;
    a2.res1 = res ? (const void*)y2 : (const void*)x1; a2.ldr1 = res ? 64 : ld1;
    RbArgs rf{};
    rf.x1 = x1; rf.ld1 = ld1; rf.C1 = q.c1; rf.x2 = x2; rf.ld2 = ld2; rf.Cin = cin; rf.B = q.B; rf.H = q.H; rf.W = q.W;
    rf.w1 = w1; rf.w2 = w2; rf.wr = res ? wr : nullptr; rf.ss = ss; rf.ss_ld = 128; rf.y = yf; rf.ldy = 64;
    dac_conv3_force(-1);
    if (res && !conv_res_fusable(a1)) { printf("%-30s no fused res_conv kernel\n", q.name); bad++; continue; }
    if (!rbfuse_ok(rf)) { printf("%-30s rbfuse_ok false\n", q.name); bad++; continue; }
    auto pair = [&]() { conv<E>(a1, 3, 3, 1, 1, 0); conv<E>(a2, 3, 3, 1, 1, 0); };
    auto fused = [&]() { rbfuse<E>(rf, 0); };
    pair(); fused();
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> hu(npx * 64), hf(npx * 64);
    CK(hipMemcpy(hu.data(), yu, npx * 128, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hf.data(), yf, npx * 128, hipMemcpyDeviceToHost));
    size_t diff = 0, first = (size_t)-1;
    for (size_t i = 0; i < hu.size(); ++i) if (hu[i] != hf[i]) { if (!diff) first = i; ++diff; }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms[2];
    for (int arm = 0; arm < 2; ++arm) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) { if (arm) fused(); else pair(); }
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[arm], e0, e1));
    }
    const double fl = 2.0 * npx * 64 * 9 * (cin + 64) + (res ? 2.0 * npx * 64 * cin : 0.0);
    printf("%s %-30s pair %7.1f us, fused %7.1f us (%6.1f TF/s)  %zu of %zu outputs differ", tn, q.name, ms[0] * 1e3 / iters,
           ms[1] * 1e3 / iters, fl / (ms[1] * 1e-3 / iters) / 1e12, diff, hu.size());
    if (diff) {
      int shown = 0;
      for (size_t i = 0; i < hu.size() && shown < 4; ++i)
        if (hu[i] != hf[i]) {
          const size_t m = i / 64;
          printf("\n    px %zu (row %zu col %zu) ch %zu: pair %04x fused %04x", m, (m / q.W) % q.H, m % q.W, i % 64, hu[i], hf[i]);
          ++shown;
        }
      printf("\n   ");
      const size_t m = first / 64;
      printf(" (first: pixel %zu (b %zu, row %zu, col %zu) ch %zu)", m, m / ((size_t)q.H * q.W), (m / q.W) % q.H, m % q.W, first % 64);
    }
    printf("  check %s\n", diff ? "FAIL" : "OK");
    bad += diff != 0;
    hipFree(x1); if (x2) hipFree(x2); hipFree(w1); hipFree(w2); hipFree(wr); hipFree(h); hipFree(y2); hipFree(yu);
    hipFree(yf); hipFree(ss); hipFree(zero);
  }
  return bad ? 1 : 0;
}

extern "C" void dac_c3i_st(int v);
// GEGLU projections on swapped tiles (ConvArgs::w_gs) against the 16-row-interleaved LDS-epilogue
// tile: the same reference weights in both orders; outputs compared element by element (max
// |diff| / max |ref|) and both forms timed (configurations 20..23 = DAC_GEGLU_SW 1..4).
static int gsw_check(int iters) {
  struct Q { const char* name; int cin, F; };
  const Q shapes[] = {{"geglu 512->2x2048", 512, 2048}, {"geglu 256->2x1024", 256, 1024}};
  const int B = 8, H = 32, W = 32;
  const size_t npx = (size_t)B * H * W;
  int bad = 0;
  for (const Q& q : shapes) {
    const int F = q.F, I = q.cin;
    std::vector<float> wr((size_t)2 * F * I), br(2 * F);
    uint32_t st = 777u;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) / 16777216.f - 0.5f); };
    for (auto& v : wr) v = 0.2f * rnd();
    for (auto& v : br) v = rnd();
    std::vector<bf16> wo((size_t)2 * F * I), wg((size_t)2 * F * I);
    std::vector<float> bo(2 * F), bg(2 * F);
    for (int r = 0; r < 2 * F; ++r) {
      const int g = r / 32, s2 = r % 32, so = s2 < 16 ? 16 * g + s2 : F + 16 * g + (s2 - 16);
      const int G = r / 64, lg = (r % 64) / 16, e = r % 16, sg = (e < 8 ? 0 : F) + 32 * G + 8 * lg + (e & 7);
      for (int k = 0; k < I; ++k) { wo[(size_t)r * I + k] = (bf16)wr[(size_t)so * I + k]; wg[(size_t)r * I + k] = (bf16)wr[(size_t)sg * I + k]; }
      bo[r] = br[so]; bg[r] = br[sg];
    }
    bf16 *x, *dwo, *dwg, *y; float *dbo, *dbg; void* zero;
    CK(hipMalloc(&x, npx * I * 2)); CK(hipMalloc(&dwo, wo.size() * 2)); CK(hipMalloc(&dwg, wg.size() * 2));
    CK(hipMalloc(&y, npx * F * 2)); CK(hipMalloc(&dbo, bo.size() * 4)); CK(hipMalloc(&dbg, bg.size() * 4));
    CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
    fill_rand<<<(npx * I + 255) / 256, 256>>>(x, npx * I, 41, 2.f);
    CK(hipMemcpy(dwo, wo.data(), wo.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwg, wg.data(), wg.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbo, bo.data(), bo.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbg, bg.data(), bg.size() * 4, hipMemcpyHostToDevice));
    ConvArgs a{};
    a.x1 = x; a.ld1 = I; a.C1 = I; a.Cin = I; a.Hs = H; a.Ws = W; a.B = B; a.Ho = H; a.Wo = W;
    a.Cout = 2 * F; a.K = I; a.w = dwo; a.bias = dbo; a.y = y; a.ldy = F; a.act = 3; a.zero = zero;
    std::vector<bf16> ref(npx * F), got(npx * F);
    auto time_it = [&]() {
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      conv<bf16>(a, 1, 1, 1, 0, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) conv<bf16>(a, 1, 1, 1, 0, 0);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1e3 / iters;
    };
    dac_conv2_force(0);
    a.w_gs = nullptr; a.b_gs = nullptr;
    const double t0 = time_it();
    CK(hipMemcpy(ref.data(), y, ref.size() * 2, hipMemcpyDeviceToHost));
    printf("%-20s LDS-epilogue tile %6.1f us", q.name, t0);
    a.w_gs = dwg; a.b_gs = dbg;
    for (int f = 20; f <= 23; ++f) {
      dac_conv2_force(f);
      CK(hipMemset(y, 0, npx * F * 2));
      const double t = time_it();
      CK(hipMemcpy(got.data(), y, got.size() * 2, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < ref.size(); ++i) { md = fmax(md, fabs((double)(float)got[i] - (float)ref[i])); mx = fmax(mx, fabs((double)(float)ref[i])); }
      const bool ok = md <= 1e-2 * mx;
      if (!ok) ++bad;
      printf("  | sw%d %6.1f us rel %.1e%s", f - 19, t, mx > 0 ? md / mx : 0.0, ok ? "" : " FAIL");
    }
    dac_conv2_force(0);
    printf("\n");
    CK(hipFree(x)); CK(hipFree(dwo)); CK(hipFree(dwg)); CK(hipFree(y)); CK(hipFree(dbo)); CK(hipFree(dbg)); CK(hipFree(zero));
  }
  printf("gsw: %s\n", bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
#ifdef DAC_STAMP
// Per-block shader-clock stamps of the 1x1 GEMM kernel (build: make convbench_stamp): where one
// launch's time goes -- first data landed, K loop, epilogue -- with warm and with flushed caches.
static int stamp_check() {
  struct Q { const char* name; int cin, cout, res, geglu; };
  const Q shapes[] = {{"1x1 512->512 +r", 512, 512, 1, 0}, {"1x1 2048->512 +r", 2048, 512, 1, 0}, {"1x1 256->256", 256, 256, 0, 0},
                      {"1x1 512->1536", 512, 1536, 0, 0}, {"1x1 512->4096 geglu", 512, 4096, 0, 1}};
  const int B = 8, H = 32, W = 32;
  const size_t npx = (size_t)B * H * W, big = (size_t)1 << 29;
  void* flush; CK(hipMalloc(&flush, big));
  for (const Q& q : shapes) {
    bf16 *x, *w, *y, *res; float* bias; void* zero; unsigned long long* st;
    CK(hipMalloc(&x, npx * q.cin * 2)); CK(hipMalloc(&w, (size_t)q.cout * q.cin * 2)); CK(hipMalloc(&y, npx * q.cout * 2));
    CK(hipMalloc(&res, npx * q.cout * 2)); CK(hipMalloc(&bias, q.cout * 4)); CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
    fill_rand<<<(npx * q.cin + 255) / 256, 256>>>(x, npx * q.cin, 31, 2.f);
    fill_rand<<<((size_t)q.cout * q.cin + 255) / 256, 256>>>(w, (size_t)q.cout * q.cin, 32, 0.1f);
    fill_rand<<<(npx * q.cout + 255) / 256, 256>>>(res, npx * q.cout, 33, 2.f);
    fill_rand_f<<<4, 256>>>(bias, q.cout, 34, 1.f);
    const int nblk = 65536;
    CK(hipMalloc(&st, (size_t)nblk * 8 * 8));
    ConvArgs a{};
    a.x1 = x; a.ld1 = q.cin; a.C1 = q.cin; a.Cin = q.cin; a.Hs = H; a.Ws = W; a.B = B; a.Ho = H; a.Wo = W;
    a.Cout = q.cout; a.K = q.cin; a.w = w; a.y = y; a.ldy = q.geglu ? q.cout / 2 : q.cout; a.bias = bias; a.zero = zero;
    if (q.geglu) a.act = 3;
    if (q.res) { a.res1 = res; a.ldr1 = q.cout; }
    for (int cold = 0; cold < 2; ++cold) {
      a.part = nullptr;
      for (int i = 0; i < 3; ++i) conv<bf16>(a, 1, 1, 1, 0, 0);
      if (cold) CK(hipMemsetAsync(flush, cold, big, 0));
      CK(hipMemset(st, 0, (size_t)nblk * 64));
      CK(hipDeviceSynchronize());
      a.part = reinterpret_cast<float*>(st);
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      if (cold) CK(hipMemsetAsync(flush, 2, big, 0));
      CK(hipEventRecord(e0, 0));
      conv<bf16>(a, 1, 1, 1, 0, 0);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> h((size_t)nblk * 8);
      CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      // s_memtime counts shader clocks of the block's own XCD (counters differ between XCDs), so
      // each block converts its intervals with its own clock: (t4 - t0) / (realtime span).
      unsigned long long r0 = ~0ull, r5 = 0;
      double first = 0, loop = 0, epi = 0, tot = 0, clk = 0, st0 = 0, setup = 0, karg = 0; int n = 0;
      for (int b = 0; b < nblk; ++b) {
        const unsigned long long* p = &h[(size_t)b * 8];
        if (!p[0] || !p[4] || p[5] <= p[1]) continue;
        ++n;
        r0 = std::min(r0, p[1]); r5 = std::max(r5, p[5]);
        const double rt = (double)(p[5] - p[1]) / 100.0;             // this block's life, us (100 MHz)
        const double c = (double)(p[4] - p[0]) / rt;                 // its clock, cycles per us
        clk += c; tot += rt;
        setup += (double)(p[6] - p[0]) / c; karg += (double)(p[7] - p[0]) / c;
        first += (double)(p[2] - p[6]) / c; loop += (double)(p[3] - p[2]) / c; epi += (double)(p[4] - p[3]) / c;
      }
      for (int b = 0; b < nblk; ++b) {
        const unsigned long long* p = &h[(size_t)b * 8];
        if (!p[0] || !p[4] || p[5] <= p[1]) continue;
        st0 += (double)(p[1] - r0) / 100.0;                           // start offset after the first block
      }
      const double us_rt = (double)(r5 - r0) / 100.0;
      printf("%-18s %s  event %6.1f us  span %6.1f us  blocks %d  clk %.2f GHz  per block: life %5.2f us (start +%5.2f)  kernarg %5.2f setup %5.2f  first data %5.2f  K loop %5.2f  epilogue %5.2f us\n",
             q.name, cold ? "cold" : "warm", ms * 1e3, us_rt, n, clk / n / 1e3, tot / n, st0 / n, karg / n, setup / n, first / n, loop / n, epi / n);
    }
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(res)); CK(hipFree(bias)); CK(hipFree(zero)); CK(hipFree(st));
  }
  return 0;
}
#endif
// Small-grid v4 ring depth (DAC_C3I_ST): time ST = 2 / 3 / 4 on the one-block-per-CU 3x3 shapes and
// require bit-identical outputs (the stage count only buffers the same ordered sum).
static int c3i_st_check(int iters) {
  struct Q { const char* name; int B, H, W, cin, cout, ss, res; };
  const Q shapes[] = {
    {"64x64 128->128 ss+silu", 8, 64, 64, 128, 128, 1, 0},
    {"64x64 128->128 silu+res", 8, 64, 64, 128, 128, 0, 1},
    {"32x32 256->256 ss+silu", 8, 32, 32, 256, 256, 1, 0},
    {"32x32 256->256 silu+res", 8, 32, 32, 256, 256, 0, 1},
  };
  int bad = 0;
  for (const Q& q : shapes) {
    const size_t npx = (size_t)q.B * q.H * q.W, nw = (size_t)q.cout * 9 * q.cin;
    bf16 *x, *w, *y, *res; float *ss, *bias; void* zero;
    CK(hipMalloc(&x, npx * q.cin * 2)); CK(hipMalloc(&w, nw * 2)); CK(hipMalloc(&y, npx * q.cout * 2));
    CK(hipMalloc(&res, npx * q.cout * 2)); CK(hipMalloc(&ss, q.B * 2 * q.cout * 4)); CK(hipMalloc(&bias, q.cout * 4));
    CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
    fill_rand<<<(npx * q.cin + 255) / 256, 256>>>(x, npx * q.cin, 21, 2.f);
    fill_rand<<<(nw + 255) / 256, 256>>>(w, nw, 22, 0.1f);
    fill_rand<<<(npx * q.cout + 255) / 256, 256>>>(res, npx * q.cout, 23, 2.f);
    fill_rand_f<<<8, 256>>>(ss, q.B * 2 * q.cout, 24, 1.f);
    fill_rand_f<<<1, 256>>>(bias, q.cout, 25, 1.f);
    ConvArgs a{};
    a.x1 = x; a.ld1 = q.cin; a.C1 = q.cin; a.Cin = q.cin; a.Hs = q.H; a.Ws = q.W; a.B = q.B; a.Ho = q.H; a.Wo = q.W;
    a.Cout = q.cout; a.K = 9 * q.cin; a.w = w; a.y = y; a.ldy = q.cout; a.act = 1; a.bias = bias; a.zero = zero;
    if (q.ss) { a.ss = ss; a.ss_ld = 2 * q.cout; }
    if (q.res) { a.res1 = res; a.ldr1 = q.cout; }
    std::vector<uint16_t> ref(npx * q.cout), got(npx * q.cout);
    printf("%-26s", q.name);
    for (int stg = 2; stg <= 4; ++stg) {
      dac_c3i_st(stg);
      dac_conv3_force(-1);
      conv<bf16>(a, 3, 3, 1, 1, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(stg == 2 ? ref.data() : got.data(), y, npx * q.cout * 2, hipMemcpyDeviceToHost));
      bool same = stg == 2 || memcmp(ref.data(), got.data(), npx * q.cout * 2) == 0;
      if (!same) ++bad;
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) conv<bf16>(a, 3, 3, 1, 1, 0);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("  ST%d %6.1f us%s", stg, ms * 1e3 / iters, same ? "" : " MISMATCH");
    }
    printf("\n");
    dac_c3i_st(2);
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(res)); CK(hipFree(ss)); CK(hipFree(bias)); CK(hipFree(zero));
  }
  printf("c3i st: %s\n", bad ? "FAIL" : "OK (bit-identical)");
  return bad ? 1 : 0;
}

template <typename E> static int conv_shapes(int argc, char** argv, const char* tn) {
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
    {"L0 4x4s2 64->64 down", 8, 256, 256, 64, 64, 4, 2, 1, 0, 0, 0, 0, 0, 1},
    {"L1 4x4s2 64->128 down", 8, 128, 128, 64, 128, 4, 2, 1, 0, 0, 0, 0, 0, 1},
    {"L2 4x4s2 128->256 down", 8, 64, 64, 128, 256, 4, 2, 1, 0, 0, 0, 0, 0, 1},
  };
  size_t maxe = (size_t)8 * 256 * 256 * 512;
  void *x, *y, *w, *res, *zero; float *ss, *bias;
  CK(hipMalloc(&x, maxe * 2)); CK(hipMalloc(&y, maxe * 2)); CK(hipMalloc(&res, maxe * 2));
  CK(hipMalloc(&w, (size_t)4096 * 9 * 1024 * 2)); CK(hipMalloc(&zero, 256));
  CK(hipMalloc(&ss, 8 * 8192 * 4)); CK(hipMalloc(&bias, 8192 * 4));
  CK(hipMemset(zero, 0, 256)); CK(hipMemset(x, 0x3c, maxe * 2)); CK(hipMemset(w, 0x3c, (size_t)4096 * 9 * 1024 * 2));
  CK(hipMemset(ss, 0, 8 * 8192 * 4)); CK(hipMemset(res, 0, maxe * 2)); CK(hipMemset(bias, 0, 8192 * 4));
  float* refo = nullptr;
  E* yh = nullptr;
  {
    // Random operands for timing too: the chip holds a lower clock on random data than on a
    // constant fill (MI355X_MICROARCH.md, DVFS give-back), so constant inputs overstate TF/s.
    const size_t nw = (size_t)4096 * 9 * 1024;
    fill_rand_t<E><<<(maxe + 255) / 256, 256>>>((E*)x, maxe, 1, 2.f);
    fill_rand_t<E><<<(nw + 255) / 256, 256>>>((E*)w, nw, 2, 0.1f);
    fill_rand_t<E><<<(maxe + 255) / 256, 256>>>((E*)res, maxe, 3, 2.f);
    fill_rand_f<<<(8 * 8192 + 255) / 256, 256>>>(ss, 8 * 8192, 4, 1.f);
    fill_rand_f<<<(8192 + 255) / 256, 256>>>(bias, 8192, 5, 1.f);
  }
  if (check) {
    CK(hipMalloc(&refo, maxe * 4));
    yh = (E*)malloc(maxe * 2);
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
    for (int i = 0; i < 3; ++i) conv<E>(a, s.kh, s.kh, s.s, s.p, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) conv<E>(a, s.kh, s.kh, s.s, s.p, 0);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double us = ms * 1e3 / iters;
    double fl = 2.0 * s.B * a.Ho * a.Wo * s.cout * s.kh * s.kh * s.cin;
    double by = 2.0 * ((double)s.B * s.H * s.W * s.cin + (double)s.B * a.Ho * a.Wo * s.cout * (1 + s.res));
    printf("%s%-26s f%-3d variant %d  %8.1f us  %7.1f TF/s  %6.0f GB/s(min bytes)", tn, s.name, force,
           conv_variant(a, s.kh, 2), us, fl / us / 1e6, by / us / 1e3);
    if (check) {
      const size_t n = (size_t)s.B * a.Ho * a.Wo * s.cout;
      ref_conv<E><<<(n + 255) / 256, 256>>>(a, s.kh, s.s, s.p, kws, refo);
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
      // Independent host (fp64) reference at 2048 sampled outputs: the operands are copied back
      // and the conv + epilogue recomputed on the CPU (the naive reference above is GPU code).
      double hd = 0, hm = 0;
      if (s.act != 3) {
        const size_t nx = (size_t)s.B * s.H * s.W * s.cin, nw = (size_t)s.cout * a.K;
        std::vector<E> hx(nx), hw(nw), hr(s.res ? n : 0);
        std::vector<float> hss(s.ss ? (size_t)s.B * 2 * s.cout : 0), hb(s.bias ? s.cout : 0);
        CK(hipMemcpy(hx.data(), x, nx * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hw.data(), w, nw * 2, hipMemcpyDeviceToHost));
        if (s.res) CK(hipMemcpy(hr.data(), res, n * 2, hipMemcpyDeviceToHost));
        if (s.ss) CK(hipMemcpy(hss.data(), ss, hss.size() * 4, hipMemcpyDeviceToHost));
        if (s.bias) CK(hipMemcpy(hb.data(), bias, hb.size() * 4, hipMemcpyDeviceToHost));
        uint32_t st = 12345u + (uint32_t)n;
        for (int q = 0; q < 2048; ++q) {
          st = st * 1664525u + 1013904223u;
          const size_t i = ((size_t)st * 2654435761u) % n;
          const int nn = (int)(i % s.cout);
          const size_t m = i / s.cout;
          const int b = (int)(m / ((size_t)a.Ho * a.Wo)), rr = (int)(m % ((size_t)a.Ho * a.Wo));
          const int oh = rr / a.Wo, ow = rr % a.Wo;
          double acc = 0;
          for (int y0 = 0; y0 < s.kh; ++y0)
            for (int z0 = 0; z0 < s.kh; ++z0) {
              const int ih = oh * s.s - s.p + y0, iw = ow * s.s - s.p + z0;
              const int Hin = s.up ? 2 * s.H : s.H, Win = s.up ? 2 * s.W : s.W;
              if (ih < 0 || iw < 0 || ih >= Hin || iw >= Win) continue;
              const int sh = s.up ? ih >> 1 : ih, sw = s.up ? iw >> 1 : iw;
              const E* xp = &hx[((size_t)(b * s.H + sh) * s.W + sw) * s.cin];
              const E* wp = &hw[(((size_t)nn * s.kh + y0) * kws + z0) * s.cin];
              for (int c = 0; c < s.cin; ++c) acc += (double)bf2f(xp[c]) * bf2f(wp[c]);
            }
          if (s.bias) acc += hb[nn];
          if (s.ss) acc = acc * (hss[(size_t)b * 2 * s.cout + nn] + 1.0) + hss[(size_t)b * 2 * s.cout + s.cout + nn];
          if (s.act == 1) acc = acc / (1.0 + std::exp(-acc));
          if (s.res) acc += bf2f(hr[m * s.cout + nn]);
          const double got = (float)yh[m * a.ldy + nn];
          hd = fmax(hd, fabs(got - acc));
          hm = fmax(hm, fabs(acc));
        }
      }
      // (GEGLU shapes: neither reference models the x * gelu(gate) pairing -- their parity is
      // covered in-network by the SpatialTransformer fixtures; timing only here.)
      if (s.act == 3) printf("  check n/a (GEGLU)");
      else {
        const bool hok = hd / hm < 1e-2;
        printf("  host rel %.2e  check rel %.2e %s", hm > 0 ? hd / hm : 0.0, md / mx, md / mx < 1e-2 && hok ? "OK" : "FAIL");
      }
    }
    printf("\n");
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "la")) return la_bench(argc > 2 ? atoi(argv[2]) : 20, argc > 3 ? atof(argv[3]) : 0.f);
  if (argc > 1 && !strcmp(argv[1], "st")) return c3i_st_check(argc > 2 ? atoi(argv[2]) : 20);
  if (argc > 1 && !strcmp(argv[1], "gsw")) return gsw_check(argc > 2 ? atoi(argv[2]) : 20);
#ifdef DAC_STAMP
  if (argc > 1 && !strcmp(argv[1], "stamp")) return stamp_check();
#endif
  if (argc > 1 && !strcmp(argv[1], "rbf")) {
    const int it = argc > 2 ? atoi(argv[2]) : 20;
    const int b = rbf_check<bf16>(it, "bf16");
    return rbf_check<_Float16>(it, "f16 ") | b;
  }
  if (argc > 1 && !strcmp(argv[1], "c3r")) return c3r_check(argc > 2 ? atoi(argv[2]) : 20);
  if (argc > 1 && !strcmp(argv[1], "fp8")) return fp8_check();
  if (argc > 1 && !strcmp(argv[1], "uph")) {
    const int it = argc > 2 ? atoi(argv[2]) : 20;
    const int b = uph_check<bf16>(it, "bf16");
    return uph_check<f16>(it, "f16 ") | b;
  }
  if (argc > 1 && !strcmp(argv[1], "q8")) return q8_check(argc > 2 ? atoi(argv[2]) : 20);
  if (argc > 1 && !strcmp(argv[1], "gns")) return gns_check();
  if (argc > 1 && !strcmp(argv[1], "lnf")) return lnf_check(argc > 2 ? atoi(argv[2]) : 20);
  // CB_DTYPE=f16: the same shapes, kernels and checks on IEEE-half operands (the bench's
  // headline dtype); default bf16.
  if (getenv("CB_DTYPE") && !strcmp(getenv("CB_DTYPE"), "f16")) return conv_shapes<f16>(argc, argv, "f16 ");
  return conv_shapes<bf16>(argc, argv, "");
}
