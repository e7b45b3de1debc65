// norm.hip — row LayerNorm and GroupNorm on NHWC activations (HBM-bound, one pass over the
// data for LayerNorm with the row held in registers; two-kernel GroupNorm).
//
// * channel LayerNorm (module_util.py:77-86): normalises over C per pixel, gain only. In NHWC
//   it is the same row operation as nn.LayerNorm over tokens (attention.py:203-205,
//   transformer.py:22-28), which adds a bias.
// * GroupNorm(32, eps=1e-6, affine) (attention.py:76-77).
#include "common.h"
#include "kernels.h"

namespace dac {

// GroupNorm statistics of the LayerNorm OUTPUT, taken by the LayerNorm kernel itself (GNS):
// the SpatialTransformer's PreNorm LN feeds its GroupNorm (attention.py:239-241), so the
// GroupNorm's pass over the data is the LN's own. Per block (one image's RPB rows) plain sums
// (sum y, sum y^2) per group, written in fixed order; the consumer (proj_in's GroupNorm-in-A
// table, conv_impl.h EPI_GNA) merges an image's blocks in fixed order. No atomics or fences:
// the kernel boundary publishes the sums. The sums are of the fp32 LayerNorm outputs, before
// their rounding to T (the separate GroupNorm pass read the rounded copy: a difference of the
// order of the storage rounding, averaged over a group).
struct GnStats { float* part; int HW, groups; };

// G lanes per row (power of two), NVL 16-byte vectors per lane.
template <typename T, int G, int NVL, bool GNS = false>
__global__ void __launch_bounds__(256) ln_kernel(const T* __restrict__ x, int ldx, T* y, int ldy,
                                                 const T* res, int ldr, const float* g,
                                                 const float* b, int rows, int C, float eps,
                                                 GnStats gs = GnStats{}) {
  constexpr int VE = TypeInfo<T>::VE;
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) + lane / G;
  const int sub = lane % G;
  const int NV = C / VE;
  float v[NVL][VE];
  float s = 0.f;
  const bool live = row < rows;
  // Gain / bias / residual loads go out with the row (they do not depend on the statistics),
  // so their latency overlaps the reductions instead of following them.
  float gv[NVL][VE], bv[NVL][VE], rv[NVL][VE];
#pragma unroll
  for (int j = 0; j < NVL; ++j) {
    const int idx = sub + G * j;
    if (live && idx < NV) {
      load_vec<T>(x + (size_t)row * ldx + idx * VE, v[j]);
      if (res) load_vec<T>(res + (size_t)row * ldr + idx * VE, rv[j]);
#pragma unroll
      for (int e = 0; e < VE; e += 4) {
        load_vec<float>(g + idx * VE + e, gv[j] + e);
        if (b) load_vec<float>(b + idx * VE + e, bv[j] + e);
      }
#pragma unroll
      for (int e = 0; e < VE; ++e) s += v[j][e];
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NVL; ++j) {
    const int idx = sub + G * j;
    if (live && idx < NV) {
#pragma unroll
      for (int e = 0; e < VE; ++e) { const float d = v[j][e] - mean; q += d * d; }
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = 1.f / sqrtf(q / (float)C + eps);
  if (!GNS && !live) return;                     // (GNS: every row is live, see layernorm_gnstats)
  float s1[NVL], s2[NVL];
#pragma unroll
  for (int j = 0; j < NVL; ++j) {
    const int idx = sub + G * j;
    s1[j] = s2[j] = 0.f;
    if (idx >= NV) continue;
    float o[VE];
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      float t = (v[j][e] - mean) * rstd * gv[j][e];
      if (b) t += bv[j][e];
      if (res) t += rv[j][e];
      o[e] = t;
      if constexpr (GNS) { s1[j] += t; s2[j] = fmaf(t, t, s2[j]); }
    }
    store_vec<T>(y + (size_t)row * ldy + idx * VE, o);
  }
  if constexpr (GNS) {
    // Group of vector idx = idx / vpg (vpg = vectors per group, divides G): sum the vpg lanes of
    // a group, then the 64 / G rows of the wave; lanes sub % vpg == 0 of row 0 hold the sums.
    const int vpg = C / gs.groups / VE;
#pragma unroll
    for (int j = 0; j < NVL; ++j) {
      for (int o = 1; o < vpg; o <<= 1) { s1[j] += __shfl_xor(s1[j], o, 64); s2[j] += __shfl_xor(s2[j], o, 64); }
#pragma unroll
      for (int o = G; o < 64; o <<= 1) { s1[j] += __shfl_xor(s1[j], o, 64); s2[j] += __shfl_xor(s2[j], o, 64); }
    }
    __shared__ float red[4][64][2];
    const int wave = threadIdx.x >> 6;
    if (lane < G && sub % vpg == 0) {
#pragma unroll
      for (int j = 0; j < NVL; ++j) {
        const int idx = sub + G * j;
        if (idx < NV) { red[wave][idx / vpg][0] = s1[j]; red[wave][idx / vpg][1] = s2[j]; }
      }
    }
    __syncthreads();
    constexpr int RPB = 4 * (64 / G);
    const int nb = gs.HW / RPB;                  // blocks per image
    const int img = (int)((long)blockIdx.x * RPB / gs.HW), blk = blockIdx.x - img * nb;
    const int t = threadIdx.x;
    if (t < gs.groups) {
      const float a0 = red[0][t][0] + red[1][t][0] + red[2][t][0] + red[3][t][0];
      const float a1 = red[0][t][1] + red[1][t][1] + red[2][t][1] + red[3][t][1];
      float* o = gs.part + (((size_t)img * gs.groups + t) * nb + blk) * 2;
      o[0] = a0; o[1] = a1;
    }
  }
}

// LayerNorm (gain, bias) whose output also yields the GroupNorm(groups) per-block sums; 16-bit
// rows of 256 or 512 channels (the SpatialTransformer widths), HW a multiple of the block's
// rows. Returns the blocks per image (the sums are part[B][groups][nb][2]), or 0 when the shape
// is not covered (the caller then runs layernorm + groupnorm_stats). launch = false only answers.
template <typename T>
int layernorm_gnstats(const void* x, int ldx, void* y, int ldy, const float* g, const float* b, int rows, int C,
                      float eps, int HW, int groups, float* part, bool launch, hipStream_t st) {
  constexpr int VE = TypeInfo<T>::VE;
  const int NV = C / VE;
#define LNG(G, NVL)                                                                                 \
  {                                                                                                 \
    constexpr int RPB = 4 * (64 / G);                                                               \
    const int vpg = groups > 0 && C % groups == 0 ? C / groups / VE : 0;                            \
    if (vpg < 1 || G % vpg || (C / groups) % VE || HW % RPB || rows % HW || groups > 64)            \
      return 0;                                                                                     \
    if (launch)                                                                                     \
      ln_kernel<T, G, NVL, true><<<rows / RPB, 256, 0, st>>>((const T*)x, ldx, (T*)y, ldy, nullptr, \
                                                             0, g, b, rows, C, eps,                 \
                                                             GnStats{part, HW, groups});            \
    return HW / RPB;                                                                                \
  }
  if (sizeof(T) == 2 && NV == 32) LNG(8, 4)
  if (sizeof(T) == 2 && NV == 64) LNG(16, 4)
#undef LNG
  return 0;
}
// Workspace floats of layernorm_gnstats (block sums), an upper bound.
size_t layernorm_gnstats_ws_floats(int B, int HW, int groups) { return (size_t)B * groups * (2 * (HW / 16) + 2); }

template <typename T>
void layernorm(const void* x, int ldx, void* y, int ldy, const void* res, int ldr,
               const float* g, const float* b, int rows, int C, float eps, hipStream_t st) {
  constexpr int VE = TypeInfo<T>::VE;
  const int NV = C / VE;
  const T* X = (const T*)x;
  T* Y = (T*)y;
  const T* R = (const T*)res;
#define LNL(G, NVL)                                                                      \
  {                                                                                      \
    const int rpb = 4 * (64 / G);                                                        \
    ln_kernel<T, G, NVL><<<(rows + rpb - 1) / rpb, 256, 0, st>>>(X, ldx, Y, ldy, R, ldr, g, \
                                                                 b, rows, C, eps);       \
    return;                                                                              \
  }
  // Up to 4 vectors per lane: more independent loads in flight per wave and shorter shuffle
  // chains than one vector per lane (the 512-wide token LNs ran at ~1 TB/s that way).
  if (NV <= 1) LNL(1, 1)
  if (NV <= 4) LNL(1, 4)
  if (NV <= 8) LNL(2, 4)
  if (NV <= 16) LNL(4, 4)
  if (NV <= 32) LNL(8, 4)
  if (NV <= 64) LNL(16, 4)
  if (NV <= 128) LNL(32, 4)
  if (NV <= 256) LNL(64, 4)
  LNL(64, 8)
#undef LNL
}

// ---------------------------------------------------------------------------- GroupNorm
// Pass 1 (gn_partial): grid (GN_CHUNKS, B). A block walks a 1/GN_CHUNKS slice of one image's
// pixels with 16-byte vector loads (thread -> fixed channel vector, pixels strided by the
// block), keeping (count, mean, M2) per thread: each vector's VE values are reduced two-pass
// in registers and merged with Chan's formula, which stays exact-ish where mean^2 >> var.
// Threads of one group are then merged in a fixed order through LDS into one partial per
// (image, chunk, group). Pass 2 (gn_apply): every thread merges its group's GN_CHUNKS
// partials in the same fixed order (identical results everywhere), then normalises its
// vector. Requires (C / groups) % VE == 0.
constexpr int GN_CHUNKS = 32;

struct Moments { float n, mean, m2; };
DEV Moments chan_merge(Moments a, Moments b) {
  const float n = a.n + b.n;
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float d = b.mean - a.mean;
  const float wb = b.n / n;
  Moments r;
  r.n = n;
  r.mean = a.mean + d * wb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * wb;
  return r;
}

template <typename T>
__global__ void __launch_bounds__(256) gn_partial(const T* __restrict__ x, float* part, int HW,
                                                  int C, int groups) {
  constexpr int VE = TypeInfo<T>::VE;
  const int b = blockIdx.y, ch = blockIdx.x;
  const int NV = C / VE;                         // vectors per pixel (<= 256)
  const int ppi = 256 / NV;                      // pixels per block iteration
  const int v = threadIdx.x % NV, p0 = threadIdx.x / NV;
  const int pbeg = (int)((long)HW * ch / GN_CHUNKS), pend = (int)((long)HW * (ch + 1) / GN_CHUNKS);
  Moments m{0.f, 0.f, 0.f};
  if (p0 < ppi) {
    const T* base = x + (size_t)b * HW * C + v * VE;
    for (int p = pbeg + p0; p < pend; p += ppi) {
      float f[VE];
      load_vec<T>(base + (size_t)p * C, f);
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < VE; ++e) s += f[e];
      const float mu = s * (1.f / VE);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < VE; ++e) { const float d = f[e] - mu; q += d * d; }
      m = chan_merge(m, Moments{(float)VE, mu, q});
    }
  }
  __shared__ float sm[3][256];
  sm[0][threadIdx.x] = m.n; sm[1][threadIdx.x] = m.mean; sm[2][threadIdx.x] = m.m2;
  __syncthreads();
  const int vpg = (C / groups) / VE;             // vectors per group
  if ((int)threadIdx.x < groups) {
    const int g = threadIdx.x;
    Moments r{0.f, 0.f, 0.f};
    for (int pp = 0; pp < ppi; ++pp)
      for (int k = 0; k < vpg; ++k) {
        const int t = pp * NV + g * vpg + k;
        r = chan_merge(r, Moments{sm[0][t], sm[1][t], sm[2][t]});
      }
    float* o = part + (((size_t)b * groups + g) * GN_CHUNKS + ch) * 3;
    o[0] = r.n; o[1] = r.mean; o[2] = r.m2;
  }
}

// Pass 2 (gn_merge): one thread per (image, group) merges its GN_CHUNKS partials in fixed
// order into (mean, rstd) at part_end = part + B * groups * GN_CHUNKS * 3.
__global__ void __launch_bounds__(64) gn_merge(float* part, int groups, float eps) {
  const int b = blockIdx.x, g = threadIdx.x;
  if (g >= groups) return;
  const float* pp = part + ((size_t)b * groups + g) * GN_CHUNKS * 3;
  float v[GN_CHUNKS * 3];                        // all loads first: one memory latency
#pragma unroll
  for (int k = 0; k < GN_CHUNKS * 3; ++k) v[k] = pp[k];
  Moments r{0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < GN_CHUNKS; ++k) r = chan_merge(r, Moments{v[3 * k], v[3 * k + 1], v[3 * k + 2]});
  float* o = part + (size_t)gridDim.x * groups * GN_CHUNKS * 3 + ((size_t)b * groups + g) * 2;
  o[0] = r.mean;
  o[1] = 1.f / sqrtf(r.m2 / r.n + eps);
}

// Pass 3 (gn_apply): y = (x - mean) * rstd * gamma + beta, one 16-byte vector per thread.
template <typename T>
__global__ void __launch_bounds__(256) gn_apply(const T* __restrict__ x, T* y,
                                                const float* stats, const float* g,
                                                const float* bta, int HW, int C, int groups,
                                                size_t nvec) {
  constexpr int VE = TypeInfo<T>::VE;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  const size_t e0 = i * VE;
  const int c0 = (int)(e0 % C);
  const int b = (int)(e0 / ((size_t)HW * C));
  const float* st = stats + ((size_t)b * groups + c0 / (C / groups)) * 2;   // one group per vector
  const float mean = st[0], rstd = st[1];
  float v[VE], gv[VE], bv[VE];
  load_vec<T>(x + e0, v);
  load_vec<float>(g + c0, gv);                   // VE floats = 1 (f32) or 2 (bf16) vectors
  load_vec<float>(bta + c0, bv);
  if constexpr (VE == 8) {
    load_vec<float>(g + c0 + 4, gv + 4);
    load_vec<float>(bta + c0 + 4, bv + 4);
  }
#pragma unroll
  for (int e = 0; e < VE; ++e) v[e] = (v[e] - mean) * rstd * gv[e] + bv[e];
  store_vec<T>(y + e0, v);
}

// Fallback for groups narrower than one vector (C / groups < VE): one block per (group,
// image), element loads, two-pass moments written as a single "chunk" (the rest zero).
template <typename T>
__global__ void __launch_bounds__(256) gn_partial_narrow(const T* __restrict__ x, float* part,
                                                         int HW, int C, int groups) {
  const int b = blockIdx.y, gi = blockIdx.x;
  const int cpg = C / groups;
  const int n = HW * cpg;
  const T* base = x + (size_t)b * HW * C + gi * cpg;
  __shared__ float red[4];
  __shared__ float s_mean;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += to_f(base[(size_t)(i / cpg) * C + i % cpg]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) s_mean = (red[0] + red[1] + red[2] + red[3]) / (float)n;
  __syncthreads();
  const float mean = s_mean;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float d = to_f(base[(size_t)(i / cpg) * C + i % cpg]) - mean;
    q += d * d;
  }
  q = wave_sum(q);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  float* o = part + ((size_t)b * groups + gi) * GN_CHUNKS * 3;
  if (threadIdx.x < GN_CHUNKS * 3) o[threadIdx.x] = 0.f;
  if (threadIdx.x == 0) { o[0] = (float)n; o[1] = mean; o[2] = red[0] + red[1] + red[2] + red[3]; }
}

template <typename T>
__global__ void __launch_bounds__(256) gn_apply_narrow(const T* __restrict__ x, T* y,
                                                       const float* part, const float* g,
                                                       const float* bta, int HW, int C,
                                                       int groups, float eps, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const int b = (int)(i / ((size_t)HW * C));
  const float* pp = part + ((size_t)b * groups + c / (C / groups)) * GN_CHUNKS * 3;
  const float rstd = 1.f / sqrtf(pp[2] / pp[0] + eps);
  y[i] = from_f<T>((to_f(x[i]) - pp[1]) * rstd * g[c] + bta[c]);
}

template <typename T>
void groupnorm(const void* x, void* y, const float* g, const float* b, int B, int HW, int C,
               int groups, float eps, float* part, hipStream_t st) {
  constexpr int VE = TypeInfo<T>::VE;
  const int NV = C / VE;
  if ((C / groups) % VE || NV > 256 || 256 % NV || groups > 64) {
    gn_partial_narrow<T><<<dim3(groups, B), 256, 0, st>>>((const T*)x, part, HW, C, groups);
    const size_t n = (size_t)B * HW * C;
    gn_apply_narrow<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const T*)x, (T*)y, part, g, b,
                                                                    HW, C, groups, eps, n);
    return;
  }
  gn_partial<T><<<dim3(GN_CHUNKS, B), 256, 0, st>>>((const T*)x, part, HW, C, groups);
  gn_merge<<<B, 64, 0, st>>>(part, groups, eps);
  const size_t nvec = (size_t)B * HW * C / TypeInfo<T>::VE;
  gn_apply<T><<<(unsigned)((nvec + 255) / 256), 256, 0, st>>>(
      (const T*)x, (T*)y, part + (size_t)B * groups * GN_CHUNKS * 3, g, b, HW, C, groups, nvec);
}

template <typename T>
const float* groupnorm_stats(const void* x, int B, int HW, int C, int groups, float eps, float* part,
                             hipStream_t st) {
  constexpr int VE = TypeInfo<T>::VE;
  const int NV = C / VE;
  if ((C / groups) % VE || NV > 256 || 256 % NV || groups > 64)   // conv_gna_ok checks this
    throw std::invalid_argument("gn: group shape not supported");
  gn_partial<T><<<dim3(GN_CHUNKS, B), 256, 0, st>>>((const T*)x, part, HW, C, groups);
  gn_merge<<<B, 64, 0, st>>>(part, groups, eps);
  return part + (size_t)B * groups * GN_CHUNKS * 3;
}

#define INST(T)                                                                              \
  template const float* groupnorm_stats<T>(const void*, int, int, int, int, float, float*, hipStream_t); \
  template int layernorm_gnstats<T>(const void*, int, void*, int, const float*, const float*, int, int, float, \
                                    int, int, float*, bool, hipStream_t);                            \
  template void layernorm<T>(const void*, int, void*, int, const void*, int, const float*,  \
                             const float*, int, int, float, hipStream_t);                   \
  template void groupnorm<T>(const void*, void*, const float*, const float*, int, int, int, \
                             int, float, float*, hipStream_t);
INST(float)
INST(bf16)
INST(f16)
#undef INST

}  // namespace dac
