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

// G lanes per row (power of two), NVL 16-byte vectors per lane.
template <typename T, int G, int NVL>
__global__ void __launch_bounds__(256) ln_kernel(const T* __restrict__ x, int ldx, T* y, int ldy,
                                                 const T* res, int ldr, const float* g,
                                                 const float* b, int rows, int C, float eps) {
  constexpr int VE = TypeInfo<T>::VE;
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) + lane / G;
  const int sub = lane % G;
  const int NV = C / VE;
  float v[NVL][VE];
  float s = 0.f;
  const bool live = row < rows;
#pragma unroll
  for (int j = 0; j < NVL; ++j) {
    const int idx = sub + G * j;
    if (live && idx < NV) {
      load_vec<T>(x + (size_t)row * ldx + idx * VE, v[j]);
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
  if (!live) return;
#pragma unroll
  for (int j = 0; j < NVL; ++j) {
    const int idx = sub + G * j;
    if (idx >= NV) continue;
    float o[VE], r[VE];
    if (res) load_vec<T>(res + (size_t)row * ldr + idx * VE, r);
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      const int c = idx * VE + e;
      float t = (v[j][e] - mean) * rstd * g[c];
      if (b) t += b[c];
      if (res) t += r[e];
      o[e] = t;
    }
    store_vec<T>(y + (size_t)row * ldy + idx * VE, o);
  }
}

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
  if (NV <= 2) LNL(2, 1)
  if (NV <= 4) LNL(4, 1)
  if (NV <= 8) LNL(8, 1)
  if (NV <= 16) LNL(16, 1)
  if (NV <= 32) LNL(32, 1)
  if (NV <= 64) LNL(64, 1)
  if (NV <= 128) LNL(64, 2)
  if (NV <= 256) LNL(64, 4)
  LNL(64, 8)
#undef LNL
}

// ---------------------------------------------------------------------------- GroupNorm
template <typename T>
__global__ void __launch_bounds__(256) gn_stats(const T* __restrict__ x, float* stats, int HW,
                                                int C, int groups, float eps) {
  const int b = blockIdx.y, gi = blockIdx.x;
  const int cpg = C / groups;
  const int n = HW * cpg;
  const T* base = x + (size_t)b * HW * C + gi * cpg;
  __shared__ float red[4];
  __shared__ float s_mean;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int p = i / cpg, c = i - p * cpg;
    s += to_f(base[(size_t)p * C + c]);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) s_mean = (red[0] + red[1] + red[2] + red[3]) / (float)n;
  __syncthreads();
  const float mean = s_mean;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int p = i / cpg, c = i - p * cpg;
    const float d = to_f(base[(size_t)p * C + c]) - mean;
    q += d * d;
  }
  q = wave_sum(q);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float var = (red[0] + red[1] + red[2] + red[3]) / (float)n;
    stats[(b * groups + gi) * 2 + 0] = mean;
    stats[(b * groups + gi) * 2 + 1] = 1.f / sqrtf(var + eps);
  }
}

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
  const int cpg = C / groups;
  float v[VE];
  load_vec<T>(x + e0, v);
#pragma unroll
  for (int e = 0; e < VE; ++e) {
    const int c = c0 + e, gi = c / cpg;
    const float* s = stats + (b * groups + gi) * 2;
    v[e] = (v[e] - s[0]) * s[1] * g[c] + bta[c];
  }
  store_vec<T>(y + e0, v);
}

template <typename T>
void groupnorm(const void* x, void* y, const float* g, const float* b, int B, int HW, int C,
               int groups, float eps, float* stats, hipStream_t st) {
  gn_stats<T><<<dim3(groups, B), 256, 0, st>>>((const T*)x, stats, HW, C, groups, eps);
  const size_t nvec = (size_t)B * HW * C / TypeInfo<T>::VE;
  gn_apply<T><<<(unsigned)((nvec + 255) / 256), 256, 0, st>>>((const T*)x, (T*)y, stats, g, b,
                                                              HW, C, groups, nvec);
}

#define INST(T)                                                                              \
  template void layernorm<T>(const void*, int, void*, int, const void*, int, const float*,  \
                             const float*, int, int, float, hipStream_t);                   \
  template void groupnorm<T>(const void*, void*, const float*, const float*, int, int, int, \
                             int, float, float*, hipStream_t);
INST(float)
INST(bf16)
#undef INST

}  // namespace dac
