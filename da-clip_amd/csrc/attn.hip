// attn.hip — self-attention kernels.
//
// flash_attn_d32: SpatialTransformer self-attention (attention.py:170-193: heads = C/32,
// d_head = 32, L = (H/8)*(W/8) tokens). Flash-style, one workgroup = 64 (or 128) queries of one
// (image, head), 4 waves x 16 queries, key tiles of 64 through LDS, online softmax in fp32.
// Computed transposed: S^T = K Q^T (A = K rows from LDS, B = this wave's 16 queries held in
// registers) and O^T = V^T P^T. Because the S^T accumulator keeps keys in registers and
// queries on lanes, P^T feeds the second MFMA straight from registers: the k order inside a
// step is permuted identically for V^T (read from LDS in that order), so no LDS round trip
// for P is needed.
//
// small_mha: nn.MultiheadAttention core of the ViT blocks (transformer.py:203, 217-230):
// L = 50 (B/32) tokens, 12 heads x 64; tiny, one workgroup per (image, head), fp32 math.
#include "common.h"
#include "kernels.h"

namespace dac {

template <typename T, int QG>
__global__ void __launch_bounds__(256) flash_d32_kernel(const T* __restrict__ qkv, T* o, int L,
                                                        int H, float scale) {
  constexpr int D = 32;
  constexpr int KT = 64;                     // keys per tile
  constexpr int ES = sizeof(T);
  constexpr int KROW = D * ES + 16;          // padded K row (bytes)
  constexpr int VROW = KT * ES + 16;         // padded V^T row (bytes)
  constexpr int KSTEP = Mma<T>::KSTEP;
  __shared__ __attribute__((aligned(16))) char sK[KT * KROW];
  __shared__ __attribute__((aligned(16))) char sV[D * VROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // XCD-aware block order: the dispatcher deals consecutive blocks to the 8 XCDs in turn, so
  // the query tiles of one (image, head) would load its K / V into 8 different L2s. Map each
  // XCD to a contiguous range of (query tile fastest, head, image) instead.
  const int gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xq = n / 8, xr = n % 8, xcd = id % 8;
  const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + id / 8;
  const int bx = t % gx, h = (t / gx) % gy, b = t / (gx * gy);
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;
  // QG groups of 16 queries per wave: every staged K/V tile and K fragment serves all of them.
  int qi[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) qi[g] = bx * (64 * QG) + wave * (16 * QG) + g * 16 + lr;

  // Q fragments (B operand of S^T = K Q^T): column = query, k = d.
  u32x4 qf[QG][D / KSTEP];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int s = 0; s < D / KSTEP; ++s) {
      const int d0 = s * KSTEP + lg * (KSTEP / 4);
      qf[g][s] = qi[g] < L ? *reinterpret_cast<const u32x4*>(base + (size_t)qi[g] * ld + h * D + d0)
                           : u32x4{0u, 0u, 0u, 0u};
    }

  f32x4 oacc[QG][2];
  float mrun[QG], lrun[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    oacc[g][0] = oacc[g][1] = f32x4{0, 0, 0, 0};
    mrun[g] = -INFINITY; lrun[g] = 0.f;
  }
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int NVEC = KT * D / VE;          // 16-byte vectors per K (or V) tile

  // K / V of the next key tile are loaded into registers while this tile computes.
  constexpr int NPT = NVEC / 256;            // vectors per thread per tile
  static_assert(NVEC % 256 == 0, "tile");
  u32x4 kreg[NPT], vreg[NPT];
  auto kv_load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int v = tid + j * 256;
      const int key = v / (D / VE), dv = (v % (D / VE)) * VE;
      const int kk = k0 + key;
      kreg[j] = vreg[j] = u32x4{0u, 0u, 0u, 0u};
      if (kk < L) {
        kreg[j] = *reinterpret_cast<const u32x4*>(base + (size_t)kk * ld + H * D + h * D + dv);
        vreg[j] = *reinterpret_cast<const u32x4*>(base + (size_t)kk * ld + 2 * H * D + h * D + dv);
      }
    }
  };
  kv_load(0);
  for (int k0 = 0; k0 < L; k0 += KT) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int v = tid + j * 256;
      const int key = v / (D / VE), dv = (v % (D / VE)) * VE;
      *reinterpret_cast<u32x4*>(sK + key * KROW + dv * ES) = kreg[j];
      const T* ve = reinterpret_cast<const T*>(&vreg[j]);
#pragma unroll
      for (int e = 0; e < VE; ++e) *reinterpret_cast<T*>(sV + (dv + e) * VROW + key * ES) = ve[e];
    }
    __syncthreads();
    if (k0 + KT < L) kv_load(k0 + KT);

#pragma unroll
    for (int g = 0; g < QG; ++g) {
      // S^T tile: 4 m-subtiles of 16 keys x this wave's 16 queries.
      f32x4 s[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        s[mi] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < D / KSTEP; ++ks) {
          const int d0 = ks * KSTEP + lg * (KSTEP / 4);
          const u32x4 ka = *reinterpret_cast<const u32x4*>(sK + (mi * 16 + lr) * KROW + d0 * ES);
          Mma<T>::run(s[mi], ka, qf[g][ks]);
        }
      }
      // Online softmax over keys for this lane's query column, in the log2 domain: the running
      // max is kept pre-scaled by c = scale * log2(e), so each probability is one FMA and one
      // v_exp_f32: p = 2^(s * c - m) (c > 0, so the max of raw scores is the max of scaled).
      const float c = scale * 1.4426950408889634f;
      float tmax = -INFINITY;
      if (k0 + KT <= L) {                        // whole tile valid (every UNet shape)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[mi][r]);
      } else {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + mi * 16 + lg * 4 + r;
            if (key >= L) s[mi][r] = -INFINITY;
            tmax = fmaxf(tmax, s[mi][r]);
          }
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(mrun[g], tmax * c);
      const float corr = sizeof(T) == 2 ? __builtin_amdgcn_exp2f(mrun[g] - mnew) : exp2f(mrun[g] - mnew);
      float psum = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = fmaf(s[mi][r], c, -mnew);
          const float p = sizeof(T) == 2 ? __builtin_amdgcn_exp2f(a) : exp2f(a);
          s[mi][r] = p;
          psum += p;
        }
      psum += __shfl_xor(psum, 16, 64);
      psum += __shfl_xor(psum, 32, 64);
      lrun[g] = lrun[g] * corr + psum;
      mrun[g] = mnew;
#pragma unroll
      for (int i = 0; i < 2; ++i) oacc[g][i] *= corr;

      // O^T += V^T P^T over the 64 keys.
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {           // k-step = 32 keys = subtiles 2st, 2st+1
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pb[j] = (bf16)s[2 * st][j];
            pb[4 + j] = (bf16)s[2 * st + 1][j];
          }
          const u32x4 pbu = __builtin_bit_cast(u32x4, pb);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const char* row = sV + (mi * 16 + lr) * VROW;
            uint2 lo = *reinterpret_cast<const uint2*>(row + (st * 32 + lg * 4) * ES);
            uint2 hi = *reinterpret_cast<const uint2*>(row + (st * 32 + 16 + lg * 4) * ES);
            Mma<T>::run(oacc[g][mi], u32x4{lo.x, lo.y, hi.x, hi.y}, pbu);
          }
        }
      } else {
#pragma unroll
        for (int st = 0; st < 4; ++st) {           // k-step = 16 keys = subtile st
          const u32x4 pbu = __builtin_bit_cast(u32x4, s[st]);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const u32x4 va = *reinterpret_cast<const u32x4*>(sV + (mi * 16 + lr) * VROW +
                                                             (st * 16 + lg * 4) * ES);
            Mma<T>::run(oacc[g][mi], va, pbu);
          }
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    if (qi[g] >= L) continue;
    const float inv = 1.f / lrun[g];
    T* out = o + ((size_t)b * L + qi[g]) * (H * D) + h * D;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[mi * 16 + lg * 4 + r] = from_f<T>(oacc[g][mi][r] * inv);
  }
}

template <typename T>
void flash_attn_d32(const void* qkv, void* o, int B, int L, int H, float scale, hipStream_t st) {
  // Two 16-query groups per wave (128 queries per block) once that still leaves >= 2 blocks
  // per CU: each staged K/V tile and its two barriers then serve twice the queries.
  if ((long)((L + 127) / 128) * H * B >= 512) {
    dim3 g((L + 127) / 128, H, B);
    flash_d32_kernel<T, 2><<<g, 256, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
  } else {
    dim3 g((L + 63) / 64, H, B);
    flash_d32_kernel<T, 1><<<g, 256, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
  }
}

// ------------------------------------------------------------------------------ small MHA
// Short-sequence MHA (ViT tokens L = 50 / 257, CLIP text L = 77), head dim 64 (or 32): one thread per
// query, K / V of the (image, head) staged in LDS as fp32, single-pass online softmax (running
// max + rescaled accumulator, so any L fits in registers); `causal` masks keys t > query
// (the text tower's additive -inf upper triangle, transformer.py:751-757).
template <typename T, int D>
__global__ void __launch_bounds__(64) small_mha_kernel(const T* __restrict__ qkv, T* o, int L, int H,
                                                       int causal) {
  extern __shared__ float sm[];               // K [L][D], V [L][D]
  const int b = blockIdx.y, h = blockIdx.x;
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;
  float* sk = sm;
  float* sv = sm + L * D;
  for (int i = threadIdx.x; i < L * (D / 4); i += 64) {
    const int t = i / (D / 4), d = (i - t * (D / 4)) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sk[t * D + d + e] = to_f(base[(size_t)t * ld + H * D + h * D + d + e]);
      sv[t * D + d + e] = to_f(base[(size_t)t * ld + 2 * H * D + h * D + d + e]);
    }
  }
  __syncthreads();
  const float scale = rsqrtf((float)D);
  for (int qi = blockIdx.z * 64 + threadIdx.x; qi < L; qi += 64 * gridDim.z) {
    float qv[D], acc[D];
#pragma unroll
    for (int d = 0; d < D; ++d) { qv[d] = to_f(base[(size_t)qi * ld + h * D + d]) * scale; acc[d] = 0.f; }
    float mx = -INFINITY, sum = 0.f;
    const int tend = causal ? qi + 1 : L;
    for (int t = 0; t < tend; ++t) {
      const float* kr = sk + t * D;
      float a = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) a += qv[d] * kr[d];
      const float mn = fmaxf(mx, a);
      const float c = expf(mx - mn), p = expf(a - mn);
      sum = sum * c + p;
      const float* vr = sv + t * D;
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = acc[d] * c + p * vr[d];
      mx = mn;
    }
    const float inv = 1.f / sum;
    T* out = o + ((size_t)b * L + qi) * (H * D) + h * D;
#pragma unroll
    for (int d = 0; d < D; ++d) out[d] = from_f<T>(acc[d] * inv);
  }
}

template <typename T>
void small_mha(const void* qkv, void* o, int B, int L, int H, int D, int causal, hipStream_t st) {
  const size_t smem = (size_t)L * 2 * D * sizeof(float);
  const dim3 g(H, B, (L + 63) / 64);
  if (D == 64) small_mha_kernel<T, 64><<<g, 64, smem, st>>>((const T*)qkv, (T*)o, L, H, causal);
  else if (D == 32) small_mha_kernel<T, 32><<<g, 64, smem, st>>>((const T*)qkv, (T*)o, L, H, causal);
  else __builtin_trap();
}

#define INST(T)                                                                           \
  template void flash_attn_d32<T>(const void*, void*, int, int, int, float, hipStream_t); \
  template void small_mha<T>(const void*, void*, int, int, int, int, int, hipStream_t);
INST(float)
INST(bf16)
#undef INST

}  // namespace dac
