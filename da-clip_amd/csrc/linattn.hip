// linattn.hip — LinearAttention context (module_util.py:157-185), heads = 4, dim_head = 32.
//
//   q = softmax_d(q) * 32^-0.5,  k = softmax_n(k),  v = v / HW
//   ctx[h][d][e] = sum_n k[h,d,n] v[h,e,n];   out = to_out(ctx^T q)
//
// The k-softmax runs over all HW pixels, so the context is a split reduction over pixel
// chunks, made exact and deterministic by taking the true per-channel max first:
//   la_kmax   : chunk-partial channel max of k                       (HBM read of k)
//   la_ctx    : per chunk, P = exp(k - max) and V staged TRANSPOSED in LDS ([ch][px]), then
//               ctx_h += P_h V_h^T on MFMA (K = pixels); exp-sums in fp32
//   la_reduce : sum the chunk partials in fixed order
//   la_weff   : W_eff[b][c][h*32+d] = sum_e Wout[c][h*32+e] ctx[h][d][e] / sum[h*32+d] / HW
// The apply step is then the to_out GEMM on softmax_d(q)*scale with per-image W_eff
// (conv.hip, amode = 1) — (Wout ctx^T) q = Wout (ctx^T q).
#include "common.h"
#include "kernels.h"

namespace dac {

constexpr int LA_PART = 4096 + 128;   // ctx + exp sums
constexpr int LA_TILE = 64;           // pixels per staged tile

// The chunking (and so the fp32 summation order of ctx) depends only on HW, never on B:
// an image restores bit-identically whatever batch / shard it is part of.
static int la_chunks(int /*B*/, int HW) {
  const int nc = 128;
  const int maxc = (HW + LA_TILE - 1) / LA_TILE;
  return nc < maxc ? nc : maxc;
}
static int la_chunk_px(int HW, int nc) {
  int ch = (HW + nc - 1) / nc;
  return (ch + LA_TILE - 1) / LA_TILE * LA_TILE;
}

size_t linear_attention_ws_floats(int B, int HW) {
  const int nc = la_chunks(B, HW);
  return (size_t)B * nc * (LA_PART + 128) + (size_t)B * LA_PART;
}

template <typename T>
__global__ void __launch_bounds__(256) la_kmax(const T* __restrict__ qkv, float* pmax, int HW,
                                               int nc, int CH) {
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int NVK = 128 / VE;           // k vectors per pixel
  constexpr int PP = 256 / NVK;           // pixels per pass
  __shared__ float red[PP][128];
  const int b = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
  const int cv = tid % NVK, pr = tid / NVK;
  const int p0 = c * CH, p1 = min(HW, p0 + CH);
  float m[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) m[e] = -INFINITY;
  const T* base = qkv + (size_t)b * HW * 384 + 128 + cv * VE;
  for (int p = p0 + pr; p < p1; p += PP) {
    float f[VE];
    load_vec<T>(base + (size_t)p * 384, f);
#pragma unroll
    for (int e = 0; e < VE; ++e) m[e] = fmaxf(m[e], f[e]);
  }
#pragma unroll
  for (int e = 0; e < VE; ++e) red[pr][cv * VE + e] = m[e];
  __syncthreads();
  if (tid < 128) {
    float r = -INFINITY;
    for (int i = 0; i < PP; ++i) r = fmaxf(r, red[i][tid]);
    pmax[((size_t)b * nc + c) * 128 + tid] = r;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) la_ctx(const T* __restrict__ qkv, const float* pmax,
                                              float* part, int HW, int nc, int CH) {
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int ES = sizeof(T);
  constexpr int ROW = LA_TILE * ES + 16;  // transposed row: one channel, 64 pixels (+pad)
  constexpr int NV2 = 256 / VE;           // vectors per pixel (k | v)
  constexpr int PP = 256 / NV2;           // pixels per pass
  constexpr int KSTEP = Mma<T>::KSTEP;
  __shared__ __attribute__((aligned(16))) char sP[128 * ROW];
  __shared__ __attribute__((aligned(16))) char sV[128 * ROW];
  __shared__ float gmax[128];
  __shared__ float sred[PP][128];

  const int b = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, h = tid >> 6, lr = lane & 15, lg = lane >> 4;
  if (tid < 128) {
    float m = -INFINITY;
    for (int i = 0; i < nc; ++i) m = fmaxf(m, pmax[((size_t)b * nc + i) * 128 + tid]);
    gmax[tid] = m;
  }
  __syncthreads();
  const int cv = tid % NV2, pr = tid / NV2;
  const bool isk = cv < NV2 / 2;
  const int c0 = (isk ? cv : cv - NV2 / 2) * VE;
  char* dst = isk ? sP : sV;
  float gm[VE], ssum[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) { gm[e] = isk ? gmax[c0 + e] : 0.f; ssum[e] = 0.f; }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  const int p0 = c * CH, p1 = min(HW, p0 + CH);
  const T* base = qkv + (size_t)b * HW * 384 + 128 + cv * VE;
  for (int t0 = p0; t0 < p1; t0 += LA_TILE) {
    __syncthreads();
    for (int pl = pr; pl < LA_TILE; pl += PP) {
      const int p = t0 + pl;
      float f[VE];
      if (p < p1) {
        load_vec<T>(base + (size_t)p * 384, f);
        if (isk) {
#pragma unroll
          for (int e = 0; e < VE; ++e) { f[e] = expf(f[e] - gm[e]); ssum[e] += f[e]; }
        }
      } else {
#pragma unroll
        for (int e = 0; e < VE; ++e) f[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < VE; ++e)
        *reinterpret_cast<T*>(dst + (c0 + e) * ROW + pl * ES) = from_f<T>(f[e]);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < LA_TILE / KSTEP; ++ks) {
      const int k0 = (ks * KSTEP + lg * (KSTEP / 4)) * ES;
      u32x4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = *reinterpret_cast<const u32x4*>(sP + (h * 32 + i * 16 + lr) * ROW + k0);
        fb[i] = *reinterpret_cast<const u32x4*>(sV + (h * 32 + i * 16 + lr) * ROW + k0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<T>::run(acc[i][j], fa[i], fb[j]);
    }
  }
  float* out = part + ((size_t)b * nc + c) * LA_PART;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(h * 32 + i * 16 + lg * 4 + r) * 32 + j * 16 + lr] = acc[i][j][r];
  __syncthreads();
  if (isk) {
#pragma unroll
    for (int e = 0; e < VE; ++e) sred[pr][c0 + e] = ssum[e];
  }
  __syncthreads();
  if (tid < 128) {
    float s = 0.f;
    for (int i = 0; i < PP; ++i) s += sred[i][tid];
    out[4096 + tid] = s;
  }
}

__global__ void __launch_bounds__(256) la_reduce(const float* part, float* ctx, int nc) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= LA_PART) return;
  const float* p = part + (size_t)b * nc * LA_PART + i;
  float s = 0.f;
  for (int c = 0; c < nc; ++c) s += p[(size_t)c * LA_PART];
  ctx[(size_t)b * LA_PART + i] = s;
}

template <typename T>
__global__ void __launch_bounds__(128) la_weff(const float* ctx, const float* wout, T* weff, int C,
                                               float inv_hw) {
  const int c = blockIdx.x, b = blockIdx.y, hd = threadIdx.x;
  const int h = hd >> 5, d = hd & 31;
  const float* cx = ctx + (size_t)b * LA_PART;
  const float* w = wout + (size_t)c * 128 + h * 32;
  float s = 0.f;
#pragma unroll 8
  for (int e = 0; e < 32; ++e) s += w[e] * cx[(h * 32 + d) * 32 + e];
  s = s / cx[4096 + hd] * inv_hw;
  weff[((size_t)b * C + c) * 128 + hd] = from_f<T>(s);
}

template <typename T>
void linear_attention_weff(const void* qkv, const float* wout, void* weff, int B, int HW, int C,
                           float* ws, hipStream_t st) {
  const int nc = la_chunks(B, HW), CH = la_chunk_px(HW, nc);
  float* part = ws;
  float* pmax = part + (size_t)B * nc * LA_PART;
  float* ctx = pmax + (size_t)B * nc * 128;
  la_kmax<T><<<dim3(nc, B), 256, 0, st>>>((const T*)qkv, pmax, HW, nc, CH);
  la_ctx<T><<<dim3(nc, B), 256, 0, st>>>((const T*)qkv, pmax, part, HW, nc, CH);
  la_reduce<<<dim3((LA_PART + 255) / 256, B), 256, 0, st>>>(part, ctx, nc);
  la_weff<T><<<dim3(C, B), 128, 0, st>>>(ctx, wout, (T*)weff, C, 1.f / (float)HW);
}

template void linear_attention_weff<float>(const void*, const float*, void*, int, int, int, float*,
                                           hipStream_t);
template void linear_attention_weff<bf16>(const void*, const float*, void*, int, int, int, float*,
                                          hipStream_t);

}  // namespace dac
