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
#include <type_traits>

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


// =====================================================================================
// Fused LinearAttention front half (PreNorm + to_qkv + context), C in {64, 128}:
//   la_proj_ctx : per (pixel chunk, image) block, one wave per head, 64-pixel tiles (32 for
//                 fp32): x tile -> channel LayerNorm in registers (module_util.py:77-86) ->
//                 LDS -> q|k|v projection on MFMA (weights in registers for bf16) ->
//                 q: softmax over the head's 32 channels * 32^-0.5, written out (the to_out
//                 GEMM reads it) ; k: online per-channel max with rescaling of the running
//                 context / sums ; exp(k - m) and v staged transposed -> ctx += P V^T (MFMA).
//   la_combine  : rescales every chunk partial to the global channel max and sums them in
//                 fixed order -> the same [ctx | sum] layout la_weff consumes.
// HBM traffic per image: read x once, write q (128 ch), instead of x->xn->qkv(384 ch)->k,v.
// The chunking depends only on HW (la_chunks), so results stay batch- and shard-invariant.
constexpr int LA_FPART = 4096 + 256;   // ctx | sum | max

// Reductions over the 16 lanes of a DPP row (the lanes holding one MFMA C-tile row): quad
// xor 1, quad xor 2, half-row mirror, row mirror -- VALU only, no LDS round trip.
template <int CTRL> DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
template <typename T> DEV float exp_t(float x);
template <> DEV float exp_t<float>(float x) { return expf(x); }
template <> DEV float exp_t<bf16>(float x) { return __expf(x); }
// bf16 handles: v_rcp_f32 / v_rsq_f32 (1 ulp) instead of the IEEE division / sqrt sequences.
template <typename T> DEV float rcp_t(float x) { return sizeof(T) == 2 ? __builtin_amdgcn_rcpf(x) : 1.f / x; }
template <typename T> DEV float rsq_t(float x) { return sizeof(T) == 2 ? __builtin_amdgcn_rsqf(x) : 1.f / sqrtf(x); }

DEV void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <typename T, int C>
struct LaCfg {
  static constexpr int ES = sizeof(T);
  static constexpr int VE = TypeInfo<T>::VE;
  static constexpr int TP = ES == 2 ? 64 : 32;           // pixels per tile
  static constexpr int PT = TP / 16;                     // 16-pixel MFMA row tiles
  static constexpr int KSTEP = Mma<T>::KSTEP;
  static constexpr int KS = C / KSTEP;                   // projection k-steps
  static constexpr int RB = C * ES;                      // x row bytes
  static constexpr int SL = RB / 16;                     // 16-byte slots per x row
  static constexpr int XT = TP * RB;                     // one x tile
  static constexpr int ROW = TP * ES + 16;               // transposed P / V row (+pad)
  static constexpr int PV = 2 * 32 * ROW;                // per wave: P and V
  static constexpr int QV = C / 4 / VE;                  // x vectors per thread (4 thr / px)
  static constexpr bool WREG = ES == 2;                  // weights cached in registers
  static constexpr int SMEM = 2 * XT + 4 * PV + 4 * 64 * 4;
  DEV static int swz(int row, int s) {                   // x tile slot swizzle
    const int f = SL >= 16 ? (row & 15) : SL == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3);
    return row * RB + ((s ^ f) << 4);
  }
};

// 16 bytes of MFMA operand (8 bf16 or 4 f32) assembled element by element.
template <typename T> struct OpPack;
template <> struct OpPack<bf16> {
  bf16x8 v;
  DEV void set(int i, float f) { v[i] = (bf16)f; }
  DEV u32x4 get() const { return __builtin_bit_cast(u32x4, v); }
};
template <> struct OpPack<float> {
  f32x4 v;
  DEV void set(int i, float f) { v[i] = f; }
  DEV u32x4 get() const { return __builtin_bit_cast(u32x4, v); }
};

template <typename T, int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C == 64 ? 2 : 1, 2))) la_proj_ctx(const T* __restrict__ x, const float* __restrict__ g,
                                                   const T* __restrict__ w, T* __restrict__ qo,
                                                   float* __restrict__ part, int HW, int nc, int CH,
                                                   float eps) {
  using K = LaCfg<T, C>;
  constexpr int VE = K::VE, TP = K::TP, PT = K::PT, KS = K::KS, KSTEP = K::KSTEP;
  __shared__ __attribute__((aligned(16))) char smem[K::SMEM];
  char* sx = smem;                                        // [2][TP][C] swizzled
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  char* sP = smem + 2 * K::XT + h * K::PV;                // this wave's [32][TP] P, then V
  float* sm = reinterpret_cast<float*>(smem + 2 * K::XT + 4 * K::PV) + h * 64;
  const int b = blockIdx.y, c = blockIdx.x;
  const int p0 = c * CH, p1 = min(HW, p0 + CH);
  float* out = part + ((size_t)b * nc + c) * LA_FPART;
  if (p0 >= p1) {                                         // empty chunk: neutral partial
    for (int i = tid; i < 4096 + 128; i += 256) out[i] = 0.f;
    if (tid < 128) out[4096 + 128 + tid] = -INFINITY;
    return;
  }
  const T* xb = x + (size_t)b * HW * C;

  // Projection weights of this head: col tile jt -> q (0,1), k (2,3), v (4,5) channels.
  auto wrow = [&](int jt) { return (jt >> 1) * 128 + h * 32 + (jt & 1) * 16 + lr; };
  u32x4 wreg[K::WREG ? 6 : 1][K::WREG ? KS : 1];
  if constexpr (K::WREG) {
#pragma unroll
    for (int jt = 0; jt < 6; ++jt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        wreg[jt][ks] = *reinterpret_cast<const u32x4*>(w + (size_t)wrow(jt) * C + ks * KSTEP + lg * (KSTEP / 4));
  }
  auto wfrag = [&](int jt, int ks) -> u32x4 {
    if constexpr (K::WREG) return wreg[jt][ks];
    else return *reinterpret_cast<const u32x4*>(w + (size_t)wrow(jt) * C + ks * KSTEP + lg * (KSTEP / 4));
  };

  // x loader: 4 threads per pixel, each C/4 channels.
  const int lp = tid >> 2, qq = tid & 3;
  u32x4 xr[K::QV];
  auto xload = [&](int t0) {
    const int p = t0 + lp;
#pragma unroll
    for (int j = 0; j < K::QV; ++j)
      xr[j] = (lp < TP && p < p1) ? *reinterpret_cast<const u32x4*>(xb + (size_t)p * C + (qq * K::QV + j) * VE)
                                  : u32x4{0u, 0u, 0u, 0u};
  };
  // LayerNorm of the loaded pixel (two-pass in registers, like ln_kernel) -> LDS tile.
  auto xstore = [&](int buf) {
    if (lp >= TP) return;
    float v[K::QV][VE];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < K::QV; ++j) {
      const T* e = reinterpret_cast<const T*>(&xr[j]);
#pragma unroll
      for (int i = 0; i < VE; ++i) { v[j][i] = to_f(e[i]); s += v[j][i]; }
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < K::QV; ++j)
#pragma unroll
      for (int i = 0; i < VE; ++i) { const float d = v[j][i] - mean; q += d * d; }
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    const float rstd = rsq_t<T>(q / (float)C + eps);
    char* dst = sx + buf * K::XT;
#pragma unroll
    for (int j = 0; j < K::QV; ++j) {
      float o[VE];
#pragma unroll
      for (int i = 0; i < VE; ++i) o[i] = (v[j][i] - mean) * rstd * g[(qq * K::QV + j) * VE + i];
      store_vec<T>(reinterpret_cast<T*>(dst + K::swz(lp, qq * K::QV + j)), o);
    }
  };

  f32x4 cacc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) cacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {-INFINITY, -INFINITY};                 // running max, k channels d = jt*16 + lr
  float srun[2] = {0.f, 0.f};                             // per-lane partial exp sums

  xload(p0);
  xstore(0);
  __syncthreads();
  int buf = 0;
  for (int t0 = p0; t0 < p1; t0 += TP) {
    const bool more = t0 + TP < p1;
    if (more) xload(t0 + TP);
    // ---- projection, in two phases to bound live accumulators: q (col tiles 0,1) first,
    // then k|v (2..5). acc[pt][jt] = xn[pt rows] . W[jt cols]
    const char* xt = sx + buf * K::XT;
    auto project = [&](auto& acc, int j0, auto nj) __attribute__((always_inline)) {
      constexpr int NJ = decltype(nj)::value;
#pragma unroll
      for (int pt = 0; pt < PT; ++pt)
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) acc[pt][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        u32x4 fa[PT];
#pragma unroll
        for (int pt = 0; pt < PT; ++pt)
          fa[pt] = *reinterpret_cast<const u32x4*>(xt + K::swz(pt * 16 + lr, ks * 4 + lg));
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) {
          const u32x4 fb = wfrag(j0 + jt, ks);
#pragma unroll
          for (int pt = 0; pt < PT; ++pt) Mma<T>::run(acc[pt][jt], fa[pt], fb);
        }
      }
    };
    f32x4 aq[PT][2];
    project(aq, 0, std::integral_constant<int, 2>{});
    // ---- q: softmax over the head's 32 channels (16 lanes x 2 tiles) per pixel row.
    T* sq = reinterpret_cast<T*>(sP);                     // [TP][32], aliases P (wave-local)
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a0 = aq[pt][0][r], a1 = aq[pt][1][r];
        const float m = row16_max(fmaxf(a0, a1));
        a0 = exp_t<T>(a0 - m);
        a1 = exp_t<T>(a1 - m);
        const float inv = rcp_t<T>(row16_sum(a0 + a1));
        const int px = pt * 16 + lg * 4 + r;
        sq[px * 32 + lr] = from_f<T>(a0 * inv * 0.17677669529663687f);
        sq[px * 32 + 16 + lr] = from_f<T>(a1 * inv * 0.17677669529663687f);
      }
    wave_sync_lds();
    {
      constexpr int CPP = 32 / VE;                        // 16-byte chunks per pixel
#pragma unroll
      for (int k = 0; k < TP * CPP / 64; ++k) {
        const int ci = lane + k * 64, px = ci / CPP, cc = (ci % CPP) * VE;
        if (t0 + px < p1)
          *reinterpret_cast<u32x4*>(qo + ((size_t)b * HW + t0 + px) * 128 + h * 32 + cc) =
              *reinterpret_cast<const u32x4*>(sq + px * 32 + cc);
      }
    }
    wave_sync_lds();
    f32x4 acc[PT][4];                                     // k (0,1) | v (2,3)
    project(acc, 2, std::integral_constant<int, 4>{});
    // ---- k: tile max per channel over valid pixels, online rescale.
    float sc[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      float m = -INFINITY;
#pragma unroll
      for (int pt = 0; pt < PT; ++pt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (t0 + pt * 16 + lg * 4 + r < p1) m = fmaxf(m, acc[pt][jt][r]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const float mn = fmaxf(mrun[jt], m);
      sc[jt] = exp_t<T>(mrun[jt] - mn);                   // 0 on the first tile
      mrun[jt] = mn;
      srun[jt] *= sc[jt];
    }
    // P = exp(k - m) and V straight from the projection accumulators: lane (lr, lg) holds
    // channel lr of pixels pt*16 + lg*4 + r, which is itself a valid MFMA operand layout
    // (row = channel, k = those pixels, the same pixel -> k map for P and V), so the context
    // MFMA needs no LDS transpose. Padding pixels are 0.
    constexpr int PPK = KSTEP / 16;                       // pixel tiles per k-step: 2 bf16, 1 f32
    static_assert(PT % PPK == 0, "pixel tiles per k-step");
    u32x4 fp[2][PT / PPK], fv[2][PT / PPK];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int kk = 0; kk < PT / PPK; ++kk) {
        OpPack<T> pp, vp;
#pragma unroll
        for (int q = 0; q < PPK; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pt = kk * PPK + q;
            const bool ok = t0 + pt * 16 + lg * 4 + r < p1;
            const float pe = ok ? exp_t<T>(acc[pt][jt][r] - mrun[jt]) : 0.f;
            srun[jt] += pe;
            pp.set(q * 4 + r, pe);
            vp.set(q * 4 + r, ok ? acc[pt][2 + jt][r] : 0.f);
          }
        fp[jt][kk] = pp.get();
        fv[jt][kk] = vp.get();
      }
    // Broadcast the per-channel rescale factors to the ctx accumulator layout (row d).
    if (lg == 0) { sm[lr] = sc[0]; sm[16 + lr] = sc[1]; }
    wave_sync_lds();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float f = sm[i * 16 + lg * 4 + r];
#pragma unroll
        for (int j = 0; j < 2; ++j) cacc[i][j][r] *= f;
      }
    // ---- ctx[d][e] += sum_px P[d][px] V[e][px]
#pragma unroll
    for (int kk = 0; kk < PT / PPK; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<T>::run(cacc[i][j], fp[i][kk], fv[j][kk]);
    wave_sync_lds();                                      // P/V reads done before next q writes
    // ---- next tile: normalise the prefetched pixels into the other buffer.
    if (more) xstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // ---- partials: ctx rows d = i*16 + lg*4 + r, cols e = j*16 + lr; sums; maxima.
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(h * 32 + i * 16 + lg * 4 + r) * 32 + j * 16 + lr] = cacc[i][j][r];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    float s = srun[jt];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lg == 0) {
      out[4096 + h * 32 + jt * 16 + lr] = s;
      out[4096 + 128 + h * 32 + jt * 16 + lr] = mrun[jt];
    }
  }
}

// ctx[b] = sum_c part_c * exp(max_c - max_g) (rows d), sums likewise. 32 elements x 8 chunk
// groups per block; the 8 group partials are combined in fixed order (deterministic).
__global__ void __launch_bounds__(256) la_combine(const float* part, float* ctx, int nc) {
  __shared__ float red[8][33];
  const int b = blockIdx.y, el = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + el;
  const bool live = i < LA_PART;
  const int d = !live ? 0 : i < 4096 ? i / 32 : i - 4096;
  const float* p = part + (size_t)b * nc * LA_FPART;
  float mg = -INFINITY;
  for (int c = grp; c < nc; c += 8) mg = fmaxf(mg, p[(size_t)c * LA_FPART + 4096 + 128 + d]);
  red[grp][el] = mg;
  __syncthreads();
  mg = red[0][el];
#pragma unroll
  for (int k = 1; k < 8; ++k) mg = fmaxf(mg, red[k][el]);
  __syncthreads();
  float s = 0.f;
  if (live)
    for (int c = grp; c < nc; c += 8) {
      const float* q = p + (size_t)c * LA_FPART;
      s += q[i] * expf(q[4096 + 128 + d] - mg);
    }
  red[grp][el] = s;
  __syncthreads();
  if (grp == 0 && live) {
    float t = red[0][el];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][el];
    ctx[(size_t)b * LA_PART + i] = t;
  }
}

size_t linear_attention_fused_ws_floats(int B, int HW) {
  const int nc = la_chunks(B, HW);
  return (size_t)B * nc * LA_FPART + (size_t)B * LA_PART;
}

template <typename T>
void linear_attention_fused(const void* x, const float* gpre, const void* wqkv, void* qout,
                            const float* wout, void* weff, int B, int HW, int C, float* ws,
                            hipStream_t st) {
  const int nc = la_chunks(B, HW), CH = la_chunk_px(HW, nc);
  float* part = ws;
  float* ctx = part + (size_t)B * nc * LA_FPART;
  if (C == 64)
    la_proj_ctx<T, 64><<<dim3(nc, B), 256, 0, st>>>((const T*)x, gpre, (const T*)wqkv, (T*)qout, part,
                                                    HW, nc, CH, 1e-5f);
  else
    la_proj_ctx<T, 128><<<dim3(nc, B), 256, 0, st>>>((const T*)x, gpre, (const T*)wqkv, (T*)qout, part,
                                                     HW, nc, CH, 1e-5f);
  la_combine<<<dim3((LA_PART + 31) / 32, B), 256, 0, st>>>(part, ctx, nc);
  la_weff<T><<<dim3(C, B), 128, 0, st>>>(ctx, wout, (T*)weff, C, 1.f / (float)HW);
}

template void linear_attention_fused<float>(const void*, const float*, const void*, void*, const float*,
                                            void*, int, int, int, float*, hipStream_t);
template void linear_attention_fused<bf16>(const void*, const float*, const void*, void*, const float*,
                                           void*, int, int, int, float*, hipStream_t);

}  // namespace dac
