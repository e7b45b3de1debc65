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
#include <algorithm>
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
// The fused pair (la_proj_ctx + la_combine_weff): fewer, longer chunks where the context pass
// is per-block-overhead bound (rocprof sweep, fp16 bench, proj + combine per launch: C = 64 at
// 256^2 41.2 -> 37.7 us with 64 chunks, C = 128 at 128^2 28.0 -> 25.0, C = 256 at 64^2 31.9 ->
// 27.3 with 32); the 512^2 levels (Wild-IR, 2 images per GPU) keep 128 to fill the chip. A
// function of (HW, C) only -- never of the batch -- and <= la_chunks() (the workspace bound).
// DAC_LA_NC overrides it (8..128, tuning).
static int la_fused_chunks(int HW, int C) {
  static const int force = getenv("DAC_LA_NC") ? atoi(getenv("DAC_LA_NC")) : 0;
  int nc = force > 0 ? (force < 8 ? 8 : force > 128 ? 128 : force) : C >= 256 ? 32 : HW >= 131072 ? 128 : 64;
  const int maxc = (HW + LA_TILE - 1) / LA_TILE;
  nc = nc < maxc ? nc : maxc;
  const int lim = la_chunks(1, HW);
  return nc < lim ? nc : lim;
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
  __shared__ float gmax[2][128];
  __shared__ float sred[PP][128];

  const int b = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, h = tid >> 6, lr = lane & 15, lg = lane >> 4;
  {
    // Global per-channel max over the chunk maxima: two threads per channel, unrolled so the
    // loads overlap (one dependent load per chunk cost ~10 us at nc = 64).
    const int ch = tid & 127, half = tid >> 7;
    float m = -INFINITY;
#pragma unroll 8
    for (int i = half; i < nc; i += 2) m = fmaxf(m, pmax[((size_t)b * nc + i) * 128 + ch]);
    gmax[half][ch] = m;
  }
  __syncthreads();
  if (tid < 128) gmax[0][tid] = fmaxf(gmax[0][tid], gmax[1][tid]);
  __syncthreads();
  const int cv = tid % NV2, pr = tid / NV2;
  const bool isk = cv < NV2 / 2;
  const int c0 = (isk ? cv : cv - NV2 / 2) * VE;
  char* dst = isk ? sP : sV;
  float gm[VE], ssum[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) { gm[e] = isk ? gmax[0][c0 + e] : 0.f; ssum[e] = 0.f; }

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

// Sum of the chunk partials: 32 elements x 8 chunk groups per block, the group sums merged
// in fixed order (deterministic; the chunking depends only on HW).
__global__ void __launch_bounds__(256) la_reduce(const float* part, float* ctx, int nc) {
  __shared__ float red[8][33];
  const int b = blockIdx.y, el = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + el;
  const bool live = i < LA_PART;
  float s = 0.f;
  if (live) {
    const float* p = part + (size_t)b * nc * LA_PART + i;
#pragma unroll 4
    for (int c = grp; c < nc; c += 8) s += p[(size_t)c * LA_PART];
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
                           float* ws, hipStream_t st, float hw_scale) {
  const int nc = la_chunks(B, HW), CH = la_chunk_px(HW, nc);
  float* part = ws;
  float* pmax = part + (size_t)B * nc * LA_PART;
  float* ctx = pmax + (size_t)B * nc * 128;
  la_kmax<T><<<dim3(nc, B), 256, 0, st>>>((const T*)qkv, pmax, HW, nc, CH);
  la_ctx<T><<<dim3(nc, B), 256, 0, st>>>((const T*)qkv, pmax, part, HW, nc, CH);
  la_reduce<<<dim3((LA_PART + 31) / 32, B), 256, 0, st>>>(part, ctx, nc);
  la_weff<T><<<dim3(C, B), 128, 0, st>>>(ctx, wout, (T*)weff, C, hw_scale > 0.f ? hw_scale : 1.f / (float)HW);
}

template void linear_attention_weff<float>(const void*, const float*, void*, int, int, int, float*,
                                           hipStream_t, float);
template void linear_attention_weff<bf16>(const void*, const float*, void*, int, int, int, float*,
                                          hipStream_t, float);
template void linear_attention_weff<f16>(const void*, const float*, void*, int, int, int, float*,
                                         hipStream_t, float);


// =====================================================================================
// Fused LinearAttention (PreNorm + to_qkv + context + to_out + LayerNorm + Residual), C in
// {64, 128}, as two passes over x (the k-softmax over all pixels forces a full-image reduction
// between them):
//   la_proj_ctx : per (pixel chunk, image) block, one wave per head, 64-pixel tiles (32 for
//                 fp32): x tile -> channel LayerNorm in registers (module_util.py:77-86) ->
//                 LDS -> k|v projection on MFMA (weights in registers for bf16) ->
//                 k: online per-channel max with rescaling of the running context / sums ;
//                 exp(k - m) and v straight from the accumulators -> ctx += P V^T (MFMA).
//   la_combine_weff : rescales every chunk partial to the global channel max, sums them in
//                 fixed order, and folds the context into per-image to_out weights
//                 W_eff = Wout ctx^T / sum / HW, written in la_apply's LDS image order.
//   la_apply    : x tile -> LayerNorm -> q projection (MFMA) -> softmax over each head's 32
//                 channels * 32^-0.5 -> out = W_eff q (MFMA, W_eff staged in LDS) -> + bias ->
//                 LayerNorm over C (to_out.1) -> + x (Residual) -> y.
// HBM traffic per image: x read twice, y written once (2 * HW * C elements in, HW * C out),
// instead of x -> xn -> qkv (384 ch) -> k, v and a q round trip. The chunking depends only
// on HW and C (la_fused_chunks), so results stay batch- and shard-invariant.
constexpr int LA_FPART = 4096 + 256;   // ctx | sum | max
// la_proj_ctx's reference-max slack (natural-log units); DAC_LA_STALE=0: -inf, the max moves on
// every tile (the exact running max of round 3).
static float la_tau() {
  static const float t = (getenv("DAC_LA_STALE") && atoi(getenv("DAC_LA_STALE")) == 0) ? -INFINITY : 5.5f;
  return t;
}

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
template <> DEV float exp_t<f16>(float x) { return __expf(x); }
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
  static constexpr int QV = C / 4 / VE;                  // x vectors per thread (4 thr / px)
  static constexpr bool WREG = ES == 2 && C <= 128;      // weights cached in registers (C = 256: L2)
  static constexpr int SMEM = 2 * XT + 4 * 64 * 4;      // x tiles + per-wave rescale scratch
  // x tile slot swizzle; thread qq of a pixel holds its 16-byte vectors qq*QV .. qq*QV + QV-1.
  // Both sides have to be conflict-free: the {lr, lg} ds_read_b128 fragment reads (16 rows from
  // a multiple of 16) and the ds_write_b128 stores (8 lanes = 2 pixels x 4 threads per group,
  // banks mod 32). 16-bit tiles: 128-byte rows s ^ (row & 7); 256/512-byte rows also fold bits
  // 3-4 of the slot into bits 1-2 before the row XOR, so a store's four slots qq*QV + j land on
  // distinct bank groups (found by enumerating both patterns; the earlier (row >> 1) & 7 and
  // row & 15 stored 2-way (C = 64, 128) and 4-way (C = 256) conflicted: SQ_LDS_BANK_CONFLICT
  // 20 % / 21 % / 47 % of the LDS cycles). Layout only: each thread keeps its channels, so its
  // LayerNorm sums are unchanged.
  DEV static int swz(int row, int s) {
    const int f = ES == 2 ? (SL == 8 ? (row & 7) : (row & 15))
                          : SL >= 16 ? (row & 15) : SL == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3);
    const int sp = ES == 2 && SL >= 16 ? s ^ (((s >> 3) & 3) << 1) : s;
    return row * RB + ((sp ^ f) << 4);
  }
  DEV static int vslot(int qq, int j) { return qq * QV + j; }
};

// 16 bytes of MFMA operand (8 bf16 or 4 f32) assembled element by element.
template <typename T> struct OpPack;
template <> struct OpPack<bf16> {
  bf16x8 v;
  DEV void set(int i, float f) { v[i] = (bf16)f; }
  DEV u32x4 get() const { return __builtin_bit_cast(u32x4, v); }
};
template <> struct OpPack<f16> {
  f16x8 v;
  DEV void set(int i, float f) { v[i] = (f16)f; }
  DEV u32x4 get() const { return __builtin_bit_cast(u32x4, v); }
};
template <> struct OpPack<float> {
  f32x4 v;
  DEV void set(int i, float f) { v[i] = f; }
  DEV u32x4 get() const { return __builtin_bit_cast(u32x4, v); }
};

template <typename T, int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C == 64 ? 2 : 1, 2))) la_proj_ctx(const T* __restrict__ x, const T* __restrict__ w,
                                                   float* __restrict__ part, int HW, int nc, int CH,
                                                   float eps, float tau) {
  using K = LaCfg<T, C>;
  constexpr int VE = K::VE, TP = K::TP, PT = K::PT, KS = K::KS, KSTEP = K::KSTEP;
  __shared__ __attribute__((aligned(16))) char smem[K::SMEM];
  char* sx = smem;                                        // [2][TP][C] swizzled
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  float* sm = reinterpret_cast<float*>(smem + 2 * K::XT) + h * 64;
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
      xr[j] = (lp < TP && p < p1) ? *reinterpret_cast<const u32x4*>(xb + (size_t)p * C + K::vslot(qq, j) * VE)
                                  : u32x4{0u, 0u, 0u, 0u};
  };
  // LayerNorm of the loaded pixel (two-pass in registers, like ln_kernel) -> LDS tile. The
  // PreNorm gain is folded into w (engine.cpp load_attn: w = to_qkv diag(g)).
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
      for (int i = 0; i < VE; ++i) o[i] = (v[j][i] - mean) * rstd;
      store_vec<T>(reinterpret_cast<T*>(dst + K::swz(lp, K::vslot(qq, j))), o);
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
    // ---- k|v projection (col tiles 2..5). acc[pt][jt] = xn[pt rows] . W[jt cols]
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
    f32x4 acc[PT][4];                                     // k (0,1) | v (2,3)
    project(acc, 2, std::integral_constant<int, 4>{});
    // ---- k: tile max per channel over valid pixels, online rescale; then P = exp(k - m) and
    // V straight from the projection accumulators: lane (lr, lg) holds channel lr of pixels
    // pt*16 + lg*4 + r, which is itself a valid MFMA operand layout (row = channel, k = those
    // pixels, the same pixel -> k map for P and V), so the context MFMA needs no LDS transpose.
    // Padding pixels are 0. Whole tiles (all but an image's last) skip the validity tests.
    // Stale reference max (16-bit types): m moves only when some k of the tile passes it by more
    // than tau (la_tau(): p = exp(k - m) <= e^5.5 fits T and the fp32 sums); the partial's max is
    // that reference, which la_combine_weff rescales like any other. Exact in m: every p and
    // every rescale of a chunk use the same m. Skips the cross-lane max, the rescale factors'
    // LDS broadcast and the context rescale on all tiles but the first (and rare movers).
    float sc[2] = {1.f, 1.f};
    bool resc = false;
    constexpr int PPK = KSTEP / 16;                       // pixel tiles per k-step: 2 bf16, 1 f32
    static_assert(PT % PPK == 0, "pixel tiles per k-step");
    u32x4 fp[2][PT / PPK], fv[2][PT / PPK];
    auto kpv = [&](auto fullc) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        float m = -INFINITY;
        if constexpr (FULL && PT % 2 == 0) {
#pragma unroll
          for (int pt = 0; pt < PT; pt += 2)
#pragma unroll
            for (int r = 0; r < 4; ++r) m = max3_raw(m, acc[pt][jt][r], acc[pt + 1][jt][r]);
        } else {
#pragma unroll
          for (int pt = 0; pt < PT; ++pt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (FULL || t0 + pt * 16 + lg * 4 + r < p1) m = fmaxf(m, acc[pt][jt][r]);
        }
        if (sizeof(T) == 4 || __any(m > mrun[jt] + tau)) {
          m = red16_max(m);
          m = red32_max(m);
          const float mn = fmaxf(mrun[jt], m);
          sc[jt] = exp_t<T>(mrun[jt] - mn);               // 0 on the first tile
          mrun[jt] = mn;
          srun[jt] *= sc[jt];
          resc = true;
        }
      }
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        // bf16: exp(k - m) = 2^(k log2e - m log2e), one v_fma + v_exp_f32.
        const float ml = mrun[jt] * 1.4426950408889634f;
#pragma unroll
        for (int kk = 0; kk < PT / PPK; ++kk) {
          OpPack<T> pp, vp;
#pragma unroll
          for (int q = 0; q < PPK; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int pt = kk * PPK + q;
              const bool ok = FULL || t0 + pt * 16 + lg * 4 + r < p1;
              float pe;
              if constexpr (sizeof(T) == 2) pe = __builtin_amdgcn_exp2f(fmaf(acc[pt][jt][r], 1.4426950408889634f, -ml));
              else pe = exp_t<T>(acc[pt][jt][r] - mrun[jt]);
              if (!FULL) pe = ok ? pe : 0.f;
              srun[jt] += pe;
              pp.set(q * 4 + r, pe);
              vp.set(q * 4 + r, ok ? acc[pt][2 + jt][r] : 0.f);
            }
          fp[jt][kk] = pp.get();
          fv[jt][kk] = vp.get();
        }
      }
    };
    if (t0 + TP <= p1) kpv(std::true_type{});
    else kpv(std::false_type{});
    // Broadcast the per-channel rescale factors to the ctx accumulator layout (row d).
    if (resc) {                                           // wave-uniform
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
      wave_sync_lds();                                    // sm reads done before the next tile
    }
    // ---- ctx[d][e] += sum_px P[d][px] V[e][px]
#pragma unroll
    for (int kk = 0; kk < PT / PPK; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<T>::run(cacc[i][j], fp[i][kk], fv[j][kk]);
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
    s = red16_sum(s);
    s = red32_sum(s);
    if (lg == 0) {
      out[4096 + h * 32 + jt * 16 + lr] = s;
      out[4096 + 128 + h * 32 + jt * 16 + lr] = mrun[jt];
    }
  }
}

// la_combine_weff: one block per (4 context rows hd0..hd0+3 of one head, image).
//  1. ctx rows: every chunk partial rescaled to the global per-row max and summed in fixed
//     order (the maxima go through LDS; 8 chunk groups x 32 columns, merged group by group),
//     likewise the exp sums -- deterministic, the chunking depends only on HW.
//  2. W_eff[c][hd] = sum_e Wout[c][h*32+e] ctx[hd][e] / sum[hd] * inv_hw for every output
//     channel c, written straight into la_apply's LDS image order (16-bit types: row
//     p = la_perm^-1(c), column k = la_qcol^-1(hd); fp32: natural [c][hd]), so la_apply
//     stages it with 16-byte copies.
template <typename T> DEV int la_prow(int c) {   // inverse of la_perm within a 64-channel half
  if constexpr (sizeof(T) == 2) {
    const int q = c & 63;
    return (c & ~63) + 32 * (q >> 5) + 16 * ((q >> 2) & 1) + 4 * ((q >> 3) & 3) + (q & 3);
  } else {
    return c;
  }
}
template <typename T> DEV int la_qcol(int qc) {  // LDS column of q channel qc in la_apply's W_eff
  if constexpr (sizeof(T) == 2) {
    const int u = qc & 31;
    return (qc & ~31) + (u < 16 ? 8 * (u >> 2) + (u & 3) : 8 * ((u - 16) >> 2) + 4 + (u & 3));
  } else {
    return qc;
  }
}

template <typename T, int NJ>   // NJ = C / 64 output (channel, row) pairs per thread, 256 at a time
__global__ void __launch_bounds__(256) la_combine_weff(const float* __restrict__ part, const float* __restrict__ wout,
                                                       T* __restrict__ weff, int C, int nc, float inv_hw) {
  constexpr int NG = 8, PER = 16;                // chunk groups x chunks per group (la_chunks() <= 128)
  __shared__ float4 sf[128];                     // per chunk: maxima of the 4 rows, then exp(max - global max)
  __shared__ float red[NG][4][33];               // group partials: 4 rows x (32 ctx + sum)
  __shared__ float4 mg2[2];
  const int b = blockIdx.y, hd0 = blockIdx.x * 4, h = hd0 >> 5;
  const int tid = threadIdx.x, grp = tid >> 5, e = tid & 31;
  const float* pb = part + (size_t)b * nc * LA_FPART;
  // Every global load is issued up front: this thread's chunk values, the sums, its Wout row
  // slices and the chunk maxima -- one memory latency for the whole kernel.
  float v[PER][4], sv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = grp + NG * k;
    const bool ok = c < nc;
    const float* pc = pb + (size_t)c * LA_FPART;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[k][r] = ok ? pc[(hd0 + r) * 32 + e] : 0.f;
    sv[k] = (ok && e < 4) ? pc[4096 + hd0 + e] : 0.f;
  }
  float4 wv[NJ][8];                              // output i = tid + 256 j: channel i >> 2
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = tid + 256 * j;
    const float* w = wout + (size_t)(i < C * 4 ? i >> 2 : 0) * 128 + h * 32;
#pragma unroll
    for (int e4 = 0; e4 < 8; ++e4) wv[j][e4] = *reinterpret_cast<const float4*>(w + 4 * e4);
  }
  float4 m = tid < nc && tid < 128 ? *reinterpret_cast<const float4*>(pb + (size_t)tid * LA_FPART + 4096 + 128 + hd0)
                                   : float4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  const float4 mine = m;
  if (tid < 128) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      m.x = fmaxf(m.x, __shfl_xor(m.x, o, 64));
      m.y = fmaxf(m.y, __shfl_xor(m.y, o, 64));
      m.z = fmaxf(m.z, __shfl_xor(m.z, o, 64));
      m.w = fmaxf(m.w, __shfl_xor(m.w, o, 64));
    }
    if ((tid & 63) == 0) mg2[tid >> 6] = m;
  }
  __syncthreads();
  if (tid < 128) {
    const float4 a0 = mg2[0], a1 = mg2[1];
    const float g[4] = {fmaxf(a0.x, a1.x), fmaxf(a0.y, a1.y), fmaxf(a0.z, a1.z), fmaxf(a0.w, a1.w)};
    const float mc[4] = {mine.x, mine.y, mine.z, mine.w};
    float f[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = mc[r] == -INFINITY ? 0.f : expf(mc[r] - g[r]);   // empty chunk: 0
    sf[tid] = float4{f[0], f[1], f[2], f[3]};
  }
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f}, sacc = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = grp + NG * k;
    if (c >= nc) break;
    const float4 f4 = sf[c];
    const float f[4] = {f4.x, f4.y, f4.z, f4.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaf(v[k][r], f[r], acc[r]);
    sacc = fmaf(sv[k], e == 0 ? f[0] : e == 1 ? f[1] : e == 2 ? f[2] : f[3], sacc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[grp][r][e] = acc[r];
  if (e < 4) red[grp][e][32] = sacc;
  __syncthreads();
  if (tid < 132) {
    const int r = tid / 33, k = tid % 33;
    float t = red[0][r][k];
#pragma unroll
    for (int g2 = 1; g2 < NG; ++g2) t += red[g2][r][k];
    red[0][r][k] = t;
  }
  __syncthreads();
  // 2. W_eff rows: thread -> (output channel c, row r).
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = tid + 256 * j;
    if (i >= C * 4) break;
    const int c = i >> 2, r = i & 3;
    float s = 0.f;
#pragma unroll
    for (int e4 = 0; e4 < 8; ++e4) {
      const float* cr = &red[0][r][4 * e4];
      s += wv[j][e4].x * cr[0] + wv[j][e4].y * cr[1] + wv[j][e4].z * cr[2] + wv[j][e4].w * cr[3];
    }
    s = s / red[0][r][32] * inv_hw;
    weff[((size_t)b * C + la_prow<T>(c)) * 128 + la_qcol<T>(hd0 + r)] = from_f<T>(s);
  }
}

size_t linear_attention_fused_ws_floats(int B, int HW) {
  const int nc = la_chunks(B, HW);
  return (size_t)B * nc * LA_FPART + (size_t)B * LA_PART;
}

// --------------------------------------------------------------------------------------
// la_apply: the back half, one wave per 16-pixel tile, no block barrier after the weight
// staging (waves walk their own tiles). Orientation is chosen so that no operand needs a
// transpose:
//   q^T[qch][px] = Wq[qch][:] . LN(x)[px][:]   A = Wq rows (LDS), B = the x tile loaded
//                                              straight from HBM in the MFMA B layout and
//                                              LayerNorm'd in registers (xor shuffles)
//   softmax over each head's 32 q channels      rows of the accumulators: registers + lanes
//   out^T[ch][px] = W_eff[ch][:] . q^T[:][px]   B = the softmaxed accumulators repacked in
//                                              registers (the k order they come in is baked
//                                              into W_eff's LDS columns), A = W_eff rows
//                                              permuted (la_perm) so each lane ends with the
//                                              very channels of its pixel it loaded for the
//                                              LayerNorm: the Residual comes from registers
//   + bias, LayerNorm over C (to_out.1), * g, + x (Residual), 16-byte stores.
// Row p = 16j + 4lg + r of a 64-channel half -> channel: bf16 32(j>>1) + 8lg + 4(j&1) + r
// (x chunk ks = 2*half + (j>>1), element 4(j&1) + r); fp32 identity (ks = 4*half + j).
template <typename T> DEV int la_perm(int p) {
  if constexpr (sizeof(T) == 2) return 32 * (p >> 5) + 8 * ((p >> 2) & 3) + 4 * ((p >> 4) & 1) + (p & 3);
  else return p;
}

// Grid (nb, B): block i of an image takes its i-th contiguous share of the image's 16-pixel
// tiles (the last one partial when HW % 16 != 0, e.g. the Wild-IR half-resolution levels),
// nb sized so the whole grid is resident at once (no half-empty second round).
template <typename T, int C>
__global__ void __launch_bounds__(256) la_apply(const T* __restrict__ x, const T* __restrict__ w,
                                                const T* __restrict__ weff,
                                                const float* __restrict__ bout, const float* __restrict__ gout,
                                                T* __restrict__ y, int HW, float eps, float wscale, float qshift) {
  constexpr int ES = sizeof(T), VE = TypeInfo<T>::VE, KSTEP = Mma<T>::KSTEP;
  constexpr int KS = C / KSTEP;                           // q-projection k-steps
  constexpr int KO = 128 / KSTEP;                         // out-GEMM k-steps
  constexpr int NH = C / 64;                              // 64-channel output halves
  // LDS rows: 128-, 256- and 512-byte rows use an XOR slot swizzle (bank-conflict free for the
  // {lr, lg} fragment reads: the +16 B padding it replaced was 2-way conflicted, 35 % of the
  // LDS cycles, and still 22 % on the C = 256 Wq rows until those took the swizzle too); wider
  // (fp32) rows keep the padding.
  constexpr int QRB = C * ES, ERB = 128 * ES;
  constexpr int WROW = (QRB == 128 || QRB == 256 || QRB == 512) ? QRB : QRB + 16;
  constexpr int EROW = (ERB == 128 || ERB == 256) ? ERB : ERB + 16;
  constexpr int SMEM = 128 * WROW + C * EROW + 2 * C * 4;
  auto qoff = [](int row, int slot) {
    if constexpr (QRB == 128) return row * 128 + ((slot ^ ((row >> 1) & 7)) << 4);
    else if constexpr (QRB == 256 || QRB == 512) return row * QRB + ((slot ^ (row & 15)) << 4);
    else return row * WROW + (slot << 4);
  };
  auto eoff = [](int row, int slot) {
    if constexpr (ERB == 128) return row * 128 + ((slot ^ ((row >> 1) & 7)) << 4);
    else if constexpr (ERB == 256) return row * 256 + ((slot ^ (row & 15)) << 4);
    else return row * EROW + (slot << 4);
  };
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  char* sq = smem;                                        // Wq [128][C]
  char* sw = smem + 128 * WROW;                           // W_eff [C][128] permuted
  float* sbo = reinterpret_cast<float*>(sw + C * EROW);   // to_out bias, then LayerNorm gain
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int nt_img = (HW + 15) / 16;
  const int p0 = (int)((long)blockIdx.x * nt_img / gridDim.x) * 16;
  const int p1 = min(HW, (int)((long)(blockIdx.x + 1) * nt_img / gridDim.x) * 16);
  if (p0 >= p1) return;
  const T* xb = x + (size_t)b * HW * C;
  T* yb = y + (size_t)b * HW * C;
  {
    // Wq = rows 0..127 of to_qkv. W_eff[b]: LDS row p of 64-half hf = channel hf*64 + perm(p);
    // column k = 32s + 8*lg' + j holds q channel rho = 32s + (j < 4 ? 4lg' + j : 16 + 4lg' + j - 4)
    // for 16-bit types (the order the repacked accumulators supply); natural order for fp32.
    // la_combine_weff writes W_eff in exactly this row / column order.
    constexpr int CPRQ = C / VE, CPRE = 128 / VE;
    for (int i = tid; i < 128 * CPRQ; i += 256) {
      const int r = i / CPRQ, cc = (i % CPRQ) * VE;
      *reinterpret_cast<u32x4*>(sq + qoff(r, cc / VE)) = *reinterpret_cast<const u32x4*>(w + (size_t)r * C + cc);
    }
    const T* wb = weff + (size_t)b * C * 128;             // already in LDS image order
    for (int i = tid; i < C * CPRE; i += 256) {
      const int p = i / CPRE, k0 = (i % CPRE) * VE;
      *reinterpret_cast<u32x4*>(sw + eoff(p, k0 / VE)) = *reinterpret_cast<const u32x4*>(wb + (size_t)p * 128 + k0);
    }
    for (int i = tid; i < 2 * C; i += 256) sbo[i] = i < C ? bout[i] : gout[i - C];
  }
  __syncthreads();

  const int ntile = (p1 - p0 + 15) / 16;
  // Two x tiles in flight per wave (tiles t + 4 and t + 8 while t is processed): the loop body
  // is written once (tile) and unrolled by 2 over the buffers xr0 / xr1.
  u32x4 xr0[KS], xr1[KS];
  auto xload = [&](u32x4 (&xr)[KS], int t) {
    const int px = p0 + t * 16 + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      xr[ks] = px < p1 ? *reinterpret_cast<const u32x4*>(xb + (size_t)px * C + ks * KSTEP + lg * VE)
                       : u32x4{0u, 0u, 0u, 0u};
  };
  auto tile = [&](u32x4 (&xr)[KS], int t) {
    // The LDS weight fragments are loop-invariant; re-read them each tile instead of letting
    // the compiler hoist ~128 VGPRs of them out of the loop (occupancy).
    asm volatile("" ::: "memory");
    // ---- LayerNorm of pixel lr (its C channels: KS*VE per lane x 4 lane groups).
    float v[KS][VE];
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const T* e = reinterpret_cast<const T*>(&xr[ks]);
#pragma unroll
      for (int j = 0; j < VE; ++j) { v[ks][j] = to_f(e[j]); s += v[ks][j]; }
    }
    s = red16_sum(s);
    s = red32_sum(s);
    const float mean = s * (1.f / (float)C);
    float qs = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < VE; ++j) { const float d = v[ks][j] - mean; qs += d * d; }
    qs = red16_sum(qs);
    qs = red32_sum(qs);
    const float rstd = rsq_t<T>(qs * (1.f / (float)C) + eps);
    u32x4 xf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      OpPack<T> pk;
#pragma unroll
      for (int j = 0; j < VE; ++j) pk.set(j, (v[ks][j] - mean) * rstd);
      xf[ks] = pk.get();
    }
    const int tcur = t;
    if (t + 8 < ntile) xload(xr, t + 8);                  // this buffer's next tile in flight
    // ---- q^T = Wq . xn^T : 8 tiles of 16 q channels.
    f32x4 aq[8];
#pragma unroll
    for (int jt = 0; jt < 8; ++jt) aq[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) {
        const u32x4 fw = *reinterpret_cast<const u32x4*>(sq + qoff(jt * 16 + lr, (ks * KSTEP + lg * VE) / VE));
        Mma<T>::run(aq[jt], fw, xf[ks]);
      }
    // ---- softmax over head hd = channels of tiles 2hd, 2hd+1 (rows 4lg + r on this lane).
#pragma unroll
    for (int hd = 0; hd < 4; ++hd) {
      // Shift: qshift > 0 bounds every q of the layer (|q_j| <= ||Wq_j|| sqrt(C), set at load
      // time only when <= 40, so exp(q - qshift) >= e^-80 stays a normal fp32 and the
      // normalised softmax is unchanged); else the per-pixel head max.
      float m = qshift;
      if (!(qshift > 0.f)) {
        m = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) m = max3_raw(m, aq[2 * hd][r], aq[2 * hd + 1][r]);
        m = red16_max(m);
        m = red32_max(m);
      }
      float sm = 0.f;
      if constexpr (ES == 2) {
        // exp(a - m) = 2^(a log2e - m log2e): one v_fma + v_exp_f32 per element.
        const float ml = m * 1.4426950408889634f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          aq[2 * hd][r] = __builtin_amdgcn_exp2f(fmaf(aq[2 * hd][r], 1.4426950408889634f, -ml));
          aq[2 * hd + 1][r] = __builtin_amdgcn_exp2f(fmaf(aq[2 * hd + 1][r], 1.4426950408889634f, -ml));
          sm += aq[2 * hd][r] + aq[2 * hd + 1][r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          aq[2 * hd][r] = exp_t<T>(aq[2 * hd][r] - m);
          aq[2 * hd + 1][r] = exp_t<T>(aq[2 * hd + 1][r] - m);
          sm += aq[2 * hd][r] + aq[2 * hd + 1][r];
        }
      }
      sm = red16_sum(sm);
      sm = red32_sum(sm);
      const float inv = rcp_t<T>(sm) * 0.17677669529663687f;
#pragma unroll
      for (int r = 0; r < 4; ++r) { aq[2 * hd][r] *= inv; aq[2 * hd + 1][r] *= inv; }
    }
    // ---- repack as B fragments of the out GEMM (k = q channel).
    u32x4 qf[KO];
#pragma unroll
    for (int s2 = 0; s2 < KO; ++s2) {
      OpPack<T> pk;
      if constexpr (ES == 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) { pk.set(r, aq[2 * s2][r]); pk.set(4 + r, aq[2 * s2 + 1][r]); }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) pk.set(r, aq[s2][r]);
      }
      qf[s2] = pk.get();
    }
    // ---- out^T = W_eff . q^T
    f32x4 acc[NH][4];
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[hf][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < KO; ++s2)
#pragma unroll
      for (int hf = 0; hf < NH; ++hf)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const u32x4 fw = *reinterpret_cast<const u32x4*>(sw + eoff(hf * 64 + j * 16 + lr, (s2 * KSTEP + lg * VE) / VE));
          Mma<T>::run(acc[hf][j], fw, qf[s2]);
        }
    // ---- epilogue: o[ks][jj] is channel ks*KSTEP + lg*VE + jj of pixel px, the element x
    // arrived in (v[ks][jj] still holds it for the Residual).
    const int px = p0 + tcur * 16 + lr;
    float o[KS][VE];
    float so = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int jj = 0; jj < VE; ++jj) {
        const int hf = ES == 2 ? ks >> 1 : ks >> 2;
        const int j = ES == 2 ? 2 * (ks & 1) + (jj >> 2) : ks & 3;
        const int r = ES == 2 ? jj & 3 : jj;
        o[ks][jj] = fmaf(acc[hf][j][r], wscale, sbo[ks * KSTEP + lg * VE + jj]);
        so += o[ks][jj];
      }
    so = red16_sum(so);
    so = red32_sum(so);
    const float mo = so * (1.f / (float)C);
    float qo = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int jj = 0; jj < VE; ++jj) { const float d = o[ks][jj] - mo; qo += d * d; }
    qo = red16_sum(qo);
    qo = red32_sum(qo);
    const float ro = rsq_t<T>(qo * (1.f / (float)C) + 1e-5f);
    if (px < p1) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float oo[VE];
#pragma unroll
        for (int jj = 0; jj < VE; ++jj)
          oo[jj] = (o[ks][jj] - mo) * ro * sbo[C + ks * KSTEP + lg * VE + jj] + v[ks][jj];
        store_vec<T>(yb + (size_t)px * C + ks * KSTEP + lg * VE, oo);
      }
    }
  };
  int t = wv;
  if (t < ntile) xload(xr0, t);
  if (t + 4 < ntile) xload(xr1, t + 4);
  for (; t < ntile; t += 8) {
    tile(xr0, t);
    if (t + 4 < ntile) tile(xr1, t + 4);
  }
}

template <typename T>
void linear_attention_fused(const void* x, const void* wqkv, const float* wout, const float* bout,
                            const float* gout, void* weff, void* y, int B, int HW, int C, float* ws,
                            hipStream_t st, float qshift) {
  const int nc = la_fused_chunks(HW, C), CH = la_chunk_px(HW, nc);
  float* part = ws;
  if (C == 64)
    la_proj_ctx<T, 64><<<dim3(nc, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, part, HW, nc, CH, 1e-5f, la_tau());
  else if (C == 128)
    la_proj_ctx<T, 128><<<dim3(nc, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, part, HW, nc, CH, 1e-5f, la_tau());
  else if constexpr (sizeof(T) == 2)
    la_proj_ctx<T, 256><<<dim3(nc, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, part, HW, nc, CH, 1e-5f, la_tau());
  else
    throw std::invalid_argument("linear attention: fp32 path supports C = 64 or 128");
  // f16: W_eff ~ |Wout ctx| / HW sits in fp16's subnormal range (~1e-5 at 256^2), so it is
  // stored without the 1/HW and la_apply applies it to the fp32 accumulators (wscale).
  const float inv_hw = 1.f / (float)HW;
  const bool hw_late = std::is_same<T, f16>::value;
  if (C == 64)
    la_combine_weff<T, 1><<<dim3(32, B), 256, 0, st>>>(part, wout, (T*)weff, C, nc, hw_late ? 1.f : inv_hw);
  else if (C == 128)
    la_combine_weff<T, 2><<<dim3(32, B), 256, 0, st>>>(part, wout, (T*)weff, C, nc, hw_late ? 1.f : inv_hw);
  else
    la_combine_weff<T, 4><<<dim3(32, B), 256, 0, st>>>(part, wout, (T*)weff, C, nc, hw_late ? 1.f : inv_hw);
  const float wscale = hw_late ? inv_hw : 1.f;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      ncu = 256;
  }
  // Resident blocks per CU (LDS-bound): 4 for 16-bit C = 64 (32 KB of weights each), 1 for
  // C = 256 (128 KB), else 2.
  const int per_cu = C == 256 ? 1 : (C == 64 && sizeof(T) == 2) ? 4 : 2;
  int nb = (per_cu * ncu + B - 1) / B;
  nb = std::max(1, std::min(nb, (HW + 63) / 64));
  if (C == 64)
    la_apply<T, 64><<<dim3(nb, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, (const T*)weff, bout, gout,
                                                 (T*)y, HW, 1e-5f, wscale, qshift);
  else if (C == 128)
    la_apply<T, 128><<<dim3(nb, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, (const T*)weff, bout, gout,
                                                  (T*)y, HW, 1e-5f, wscale, qshift);
  else if constexpr (sizeof(T) == 2)
    la_apply<T, 256><<<dim3(nb, B), 256, 0, st>>>((const T*)x, (const T*)wqkv, (const T*)weff, bout, gout,
                                                  (T*)y, HW, 1e-5f, wscale, qshift);
}

template void linear_attention_fused<float>(const void*, const void*, const float*, const float*, const float*,
                                            void*, void*, int, int, int, float*, hipStream_t, float);
template void linear_attention_fused<bf16>(const void*, const void*, const float*, const float*, const float*,
                                            void*, void*, int, int, int, float*, hipStream_t, float);
template void linear_attention_fused<f16>(const void*, const void*, const float*, const float*, const float*,
                                            void*, void*, int, int, int, float*, hipStream_t, float);

}  // namespace dac
