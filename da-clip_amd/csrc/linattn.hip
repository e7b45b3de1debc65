// linattn.hip — LinearAttention (module_util.py:157-185), heads = 4, dim_head = 32.
//
//   q = softmax_d(q) * 32^-0.5,  k = softmax_n(k),  v = v / HW
//   ctx[h][d][e] = sum_n k[h,d,n] v[h,e,n]          (32x32 per head)
//   out[h*32+e, n] = sum_d ctx[h][d][e] q[h,d,n]
//
// The k-softmax runs over all HW pixels, so the context is a split reduction:
//   la_partial : per (image, chunk of LA_CHUNK pixels), online max / exp-sum / k v^T with
//                rescaling across 64-pixel sub-tiles staged in LDS;
//   la_combine : per image, merge the chunk partials (rescale by exp(max_c - max));
//   la_apply   : per (pixel, head) q-softmax and the 32x32 context product.
// qkv rows are [q(128) | k(128) | v(128)] (the to_qkv 1x1 conv output, channels-last).
#include "common.h"
#include "kernels.h"

namespace dac {

constexpr int LA_CHUNK = 1024;
constexpr int LA_SUB = 64;
constexpr int LA_PART = 128 + 128 + 4096;    // max, sum, ctx

size_t linear_attention_ws_floats(int B, int HW) {
  const int nc = (HW + LA_CHUNK - 1) / LA_CHUNK;
  return (size_t)B * nc * LA_PART + (size_t)B * 4096;
}

template <typename T>
__global__ void __launch_bounds__(256) la_partial(const T* __restrict__ qkv, float* part, int HW,
                                                  int nc) {
  __shared__ float sk[LA_SUB][129];
  __shared__ float sv[LA_SUB][129];
  __shared__ float smax[128], ssum[128], snew[128];
  const int b = blockIdx.y, c = blockIdx.x;
  const int tid = threadIdx.x;
  const int p0 = c * LA_CHUNK, p1 = min(HW, p0 + LA_CHUNK);
  if (tid < 128) { smax[tid] = -INFINITY; ssum[tid] = 0.f; }
  // Each thread owns 16 ctx entries: head h, row d, columns e0..e0+15.
  const int h = tid >> 6, d = (tid >> 1) & 31, e0 = (tid & 1) * 16;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const T* base = qkv + (size_t)b * HW * 384;
  for (int s0 = p0; s0 < p1; s0 += LA_SUB) {
    const int ns = min(LA_SUB, p1 - s0);
    __syncthreads();
    for (int i = tid; i < LA_SUB * 256; i += 256) {
      const int p = i >> 8, ch = i & 255;
      float v = 0.f;
      if (p < ns) v = to_f(base[(size_t)(s0 + p) * 384 + 128 + ch]);
      if (ch < 128) sk[p][ch] = v; else sv[p][ch - 128] = v;
    }
    __syncthreads();
    if (tid < 128) {
      float m = smax[tid];
      for (int p = 0; p < ns; ++p) m = fmaxf(m, sk[p][tid]);
      const float corr = expf(smax[tid] - m);
      float s = ssum[tid] * corr;
      for (int p = 0; p < ns; ++p) {
        const float e = expf(sk[p][tid] - m);
        sk[p][tid] = e;
        s += e;
      }
      snew[tid] = corr;
      smax[tid] = m;
      ssum[tid] = s;
    }
    __syncthreads();
    const float corr = snew[h * 32 + d];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] *= corr;
    for (int p = 0; p < ns; ++p) {
      const float kv = sk[p][h * 32 + d];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] += kv * sv[p][h * 32 + e0 + i];
    }
  }
  __syncthreads();
  float* out = part + ((size_t)b * nc + c) * LA_PART;
  if (tid < 128) { out[tid] = smax[tid]; out[128 + tid] = ssum[tid]; }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[256 + (h * 32 + d) * 32 + e0 + i] = acc[i];
}

__global__ void __launch_bounds__(256) la_combine(const float* part, float* ctx, int HW, int nc) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ float gmax[128], gsum[128];
  const float* pb = part + (size_t)b * nc * LA_PART;
  if (tid < 128) {
    float m = -INFINITY;
    for (int c = 0; c < nc; ++c) m = fmaxf(m, pb[(size_t)c * LA_PART + tid]);
    float s = 0.f;
    for (int c = 0; c < nc; ++c)
      s += pb[(size_t)c * LA_PART + 128 + tid] * expf(pb[(size_t)c * LA_PART + tid] - m);
    gmax[tid] = m;
    gsum[tid] = s;
  }
  __syncthreads();
  for (int i = tid; i < 4096; i += 256) {
    const int ch = i >> 5;   // h*32 + d
    float s = 0.f;
    for (int c = 0; c < nc; ++c)
      s += pb[(size_t)c * LA_PART + 256 + i] * expf(pb[(size_t)c * LA_PART + ch] - gmax[ch]);
    ctx[(size_t)b * 4096 + i] = s / gsum[ch] / (float)HW;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) la_apply(const T* __restrict__ qkv, const float* ctx,
                                                T* out, int B, int HW) {
  __shared__ float sc[4096];
  const int tid = threadIdx.x;
  const int h = tid & 3;
  const size_t n = (size_t)blockIdx.x * 64 + (tid >> 2);
  const size_t N = (size_t)B * HW;
  const int b0 = (int)(((size_t)blockIdx.x * 64) / HW);
  const size_t nlast = min(N, (size_t)blockIdx.x * 64 + 64) - 1;
  const bool uni = (int)(nlast / HW) == b0;
  if (uni) {
    for (int i = tid; i < 4096; i += 256) sc[i] = ctx[(size_t)b0 * 4096 + i];
    __syncthreads();
  }
  if (n >= N) return;
  const float* cx = uni ? sc : ctx + (n / HW) * 4096;
  float q[32];
  const T* qp = qkv + n * 384 + h * 32;
  float m = -INFINITY;
#pragma unroll
  for (int d = 0; d < 32; ++d) { q[d] = to_f(qp[d]); m = fmaxf(m, q[d]); }
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < 32; ++d) { q[d] = expf(q[d] - m); s += q[d]; }
  const float inv = 1.f / s;
  const float scale = 0.17677669529663687f;   // 32^-0.5
#pragma unroll
  for (int d = 0; d < 32; ++d) q[d] = q[d] * inv * scale;
  T* op = out + n * 128 + h * 32;
  const float* ch = cx + h * 1024;
  for (int e = 0; e < 32; ++e) {
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) a += ch[d * 32 + e] * q[d];
    op[e] = from_f<T>(a);
  }
}

template <typename T>
void linear_attention(const void* qkv, void* out, int B, int HW, float* ws, hipStream_t st) {
  const int nc = (HW + LA_CHUNK - 1) / LA_CHUNK;
  float* part = ws;
  float* ctx = ws + (size_t)B * nc * LA_PART;
  la_partial<T><<<dim3(nc, B), 256, 0, st>>>((const T*)qkv, part, HW, nc);
  la_combine<<<B, 256, 0, st>>>(part, ctx, HW, nc);
  const size_t N = (size_t)B * HW;
  la_apply<T><<<(unsigned)((N + 63) / 64), 256, 0, st>>>((const T*)qkv, ctx, (T*)out, B, HW);
}

template void linear_attention<float>(const void*, void*, int, int, float*, hipStream_t);
template void linear_attention<bf16>(const void*, void*, int, int, float*, hipStream_t);

}  // namespace dac
