// conv_impl.h — MFMA implicit-GEMM convolution kernels for gfx950 (NHWC activations).
//
// One kernel covers every conv/linear of the hot path (SURVEY.md §2.3 op census):
// conv3x3 s1 p1 (module_util.py:111-112), conv4x4 s2 p1 (Downsample, :107-108),
// nearest-2x + conv3x3 (Upsample, :100-104), conv7x7 (init_conv), 1x1 convs / nn.Linear
// (to_qkv, res_conv, proj_in/out, q/k/v/out, GEGLU, ViT projections) and the ViT 32x32/s32
// patch embedding (transformer.py:411).
//
// Tiling: 256 threads = 4 waves arranged WGM x WGN over a BM x BN output tile; each wave owns
// a (BM/WGM) x (BN/WGN) sub-tile of 16x16 MFMA tiles. The K loop walks 128-byte K slices
// (64 bf16 or 32 f32 per row) through double-buffered LDS; global->register prefetch of
// slice k+1 overlaps the MFMAs of slice k. LDS rows are 128 B with the 16-byte slot
// XOR-swizzled by (row>>1)&7 so the 16 rows read by a ds_read_b128 lane group hit distinct
// banks.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "common.h"
#include "kernels.h"
#include "conv_epi.h"

namespace dac {

// XCD-aware block order (cdna_hip_programming.md T1): the dispatcher deals blocks round-robin
// over the 8 XCDs, so neighbouring output tiles (which share input rows / weights) would
// sit in different L2s. Remap the linear block id bijectively so each XCD walks a
// contiguous range of (n-tile fastest, then m-tile, then image) tiles. Speed only.
struct TileId { int bx, by, bz; };
DEV TileId xcd_tile() {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int n = gx * gy * gz;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int q = n / 8, r = n % 8, xcd = id % 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
  TileId o;
  o.by = t % gy;
  o.bx = (t / gy) % gx;
  o.bz = t / (gy * gx);
  return o;
}

template <typename T, int BM, int BN, int WGM, int WGN, int KH, int KW, int S, int P>
__global__ void __launch_bounds__(256) conv_kernel(ConvArgs a) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int BKE = 128 / sizeof(T);
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int AV = BM / 32;
  constexpr int BV = (BN + 31) / 32;
  constexpr int KSTEPS = BKE / Mma<T>::KSTEP;
  static_assert(WGM * WGN == 4 && TM >= 1 && TN >= 1, "tile");
  constexpr int PIPE = 2 * (BM + BN) * 128;
  constexpr int EPR = epi_rows<BM, BN, WTM>(PIPE);
  constexpr int SMEM = PIPE > EpiLds<EPR, BN>::BYTES ? PIPE : EpiLds<EPR, BN>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int HWo = a.Ho * a.Wo;
  const TileId tl = xcd_tile();
  // Batched grid (per-image weights): rows of image tl.bz only.
  const bool batched = a.w_bstride > 0;
  const int M = batched ? (tl.bz + 1) * HWo : a.B * HWo;
  const int m0 = (batched ? tl.bz * HWo : 0) + tl.bx * BM, n0 = tl.by * BN;
  const int slot = tid & 7, rbase = tid >> 3;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;

  // Per-thread A rows: output pixel -> (image base, top-left input coordinate).
  int a_pix[AV], a_ih[AV], a_iw[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    int m = m0 + rbase + 32 * i;
    if (m < M) {
      int b = m / HWo, r = m - b * HWo;
      int oh = r / a.Wo, ow = r - oh * a.Wo;
      a_pix[i] = b * a.Hs * a.Ws;
      a_ih[i] = oh * S - P;
      a_iw[i] = ow * S - P;
    } else {
      a_pix[i] = 0; a_ih[i] = -100000; a_iw[i] = -100000;
    }
  }
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  const T* wgt = reinterpret_cast<const T*>(a.w) + (batched ? tl.bz * a.w_bstride : 0);

  u32x4 ra[AV], rb[BV];
  const int nk = (a.K + BKE - 1) / BKE;

  auto gload = [&](int kt) {
    const int k = kt * BKE + slot * VE;
    const bool kv = k < a.K;
    int kpos = k / a.Cin;
    int ci = k - kpos * a.Cin;
    if (a.cwrap && ci >= a.cwrap) ci -= a.cwrap;
    const int kh = kpos / KW, kw = kpos - (kpos / KW) * KW;
    const bool from1 = ci < a.C1;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int ih = a_ih[i] + kh, iw = a_iw[i] + kw;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kv && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win) {
        const int sh = a.up ? (ih >> 1) : ih, sw = a.up ? (iw >> 1) : iw;
        const size_t pix = (size_t)(a_pix[i] + sh * a.Ws + sw);
        const T* src = from1 ? x1 + pix * a.ld1 + ci : x2 + pix * a.ld2 + (ci - a.C1);
        v = *reinterpret_cast<const u32x4*>(src);
      }
      ra[i] = v;
    }
    if (a.amode == 1) {
      // softmax over the 32 channels of each head (32/VE lanes of one row share a head).
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        float f[VE];
        const T* e = reinterpret_cast<const T*>(&ra[i]);
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < VE; ++j) { f[j] = to_f(e[j]); mx = fmaxf(mx, f[j]); }
#pragma unroll
        for (int o = 1; o < 32 / VE; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < VE; ++j) { f[j] = expf(f[j] - mx); sm += f[j]; }
#pragma unroll
        for (int o = 1; o < 32 / VE; o <<= 1) sm += __shfl_xor(sm, o, 64);
        const float inv = 1.f / sm;
        T* w = reinterpret_cast<T*>(&ra[i]);
#pragma unroll
        for (int j = 0; j < VE; ++j) w[j] = from_f<T>(f[j] * inv * 0.17677669529663687f);
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int r = rbase + 32 * i;
      const int n = n0 + r;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r < BN && n < a.Cout && kv) v = *reinterpret_cast<const u32x4*>(wgt + (size_t)n * a.K + k);
      rb[i] = v;
    }
  };
  auto swz = [](int row, int s) { return row * 128 + ((s ^ ((row >> 1) & 7)) << 4); };
  auto swrite = [&](int buf) {
    char* A = smem + buf * (BM + BN) * 128;
    char* Bs = A + BM * 128;
#pragma unroll
    for (int i = 0; i < AV; ++i) *reinterpret_cast<u32x4*>(A + swz(rbase + 32 * i, slot)) = ra[i];
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int r = rbase + 32 * i;
      if (r < BN) *reinterpret_cast<u32x4*>(Bs + swz(r, slot)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  swrite(0);
  __syncthreads();
  const int lr = lane & 15, lg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* A = smem + cur * (BM + BN) * 128;
    const char* Bs = A + BM * 128;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      u32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const u32x4*>(A + swz(wm * WTM + i * 16 + lr, ks * 4 + lg));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const u32x4*>(Bs + swz(wn * WTN + j * 16 + lr, ks * 4 + lg));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Mma<T>::run(acc[i][j], fa[i], fb[j]);
    }
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;
  const int bimg = (m0 / HWo == mlast / HWo) ? m0 / HWo : -1;
  conv_epilogue_lds<T, BM, BN, WGM, WGN, EPR>(a, acc, smem, M, LinearRows{m0}, n0, HWo, bimg);
}


// Register epilogue of the swapped-operand 16-bit tiles (weights as the MFMA A operand, weight
// row p holding output channel 16*((p>>2)&3) + 4*(p>>4) + (p&3) of its 64-channel tile):
// acc[i][j][r] is channel nb + 4j + r of output row pix(i), nb = tile base + 16*(lane>>4), so
// each lane finishes 16 consecutive channels with 16-byte loads and stores, no LDS staging.
// EPI_MIN order: (acc + bias) * (1 + scale) + shift -> SiLU -> + res1 + res2 + bbias.
// All residual rows are requested first, so their latency overlaps the SiLU math.
DEV int wperm64(int p) { return 16 * ((p >> 2) & 3) + 4 * (p >> 4) + (p & 3); }
// LN = true (to_out of LinearAttention, Cout = 64 in one wave): row LayerNorm over the 64
// channels held by lanes lr, lr+16, lr+32, lr+48 (two xor shuffles), gain ln_g, after the bias
// and before the residual (module_util.py:77-86, 180-185).
// Operands of a register epilogue loaded ahead: a persistent kernel issues them before the
// next tile's first DMA, so waiting for them never waits for that DMA (vmcnt retires in issue
// order). One register set holds either the residual rows (res1) or, on convs without one,
// the per-image scale/shift rows (ss) — the UNet's block2 and block1 convs respectively.
template <int TM> struct EpiPref { u32x4 v[2 * TM > 8 ? 2 * TM : 8]; };
// The loads are inline asm the compiler cannot see: its wait insertion treats vmcnt as out of
// order once loads, stores and LDS-DMA are all pending, and would put a vmcnt(0) — a wait for
// the next tile's DMA too — ahead of the first use. The caller waits with a counted vmcnt
// instead (these loads are older than every DMA issued after them), before any use.
DEV void ld_asm(u32x4& r, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
}
template <typename T, int TM, class PixOf>
DEV void epi_prefetch(const ConvArgs& a, int nb, int b, const PixOf& pix, EpiPref<TM>& p) {
  // One set of loads whatever the operand (addresses selected, not branches): per-branch
  // destinations would be merged by register copies, reading registers still in flight.
  constexpr int N = 2 * TM > 8 ? 2 * TM : 8;
  if (!a.res1 && !a.ss) return;
  const T* r1 = reinterpret_cast<const T*>(a.res1);
  const float* s4 = a.ss + (size_t)b * a.ss_ld + nb;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int i = k / 2 < TM ? k / 2 : TM - 1, q = k & 7;
    const void* src = r1 ? (const void*)(r1 + pix(i) * a.ldr1 + nb + 8 * (k & 1))
                         : (const void*)(s4 + (q < 4 ? 4 * q : a.Cout + 4 * (q - 4)));
    ld_asm(p.v[k], src);
  }
}

typedef short short2_t __attribute__((ext_vector_type(2)));
// fp8 output of a register epilogue (ConvArgs::ys8): the lane's 16 values of pixel m, channels
// nb .. nb+15, become e4m3 under one E8M0 exponent per 32-channel half (lanes lg and lg ^ 1 hold
// one half: a permlane16 max). The exponent is the smallest with |v| / 2^e <= 440 (a margin below
// e4m3's 448, so the product rounding of max / 440 can never push a value past it); one 16-byte
// store of the bytes, one byte store of the exponent from the half's first lane.
DEV void q8_store(const ConvArgs& a, size_t m, int nb, const float (&v)[16]) {
  float mx = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) mx = fmaxf(mx, fabsf(v[e]));
  mx = red16_max(mx);
  const uint32_t u = __float_as_uint(mx * (1.f / 440.f));
  int ex = (int)(u >> 23) - 127 + ((u & 0x7fffffu) != 0u);
  ex = ex < -126 ? -126 : (ex > 126 ? 126 : ex);
  const float sc = __uint_as_float((uint32_t)(ex + 127) << 23);
  u32x4 q;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    short2_t s = {0, 0};
    s = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s, v[4 * w], v[4 * w + 1], sc, false);
    s = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s, v[4 * w + 2], v[4 * w + 3], sc, true);
    q[w] = __builtin_bit_cast(uint32_t, s);
  }
  *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(a.y) + m * a.ldy + nb) = q;
  if ((nb & 16) == 0) a.ys8[m * (a.Cout >> 5) + (nb >> 5)] = (uint8_t)(ex + 127);
}

// PRE: operands come from epi_prefetch and the conv has no bbias / res2 / (ss with res1) —
// the epilogue then issues no loads at all, so it never waits for in-flight DMA.
// Q8: the output is e4m3 + exponents (q8_store) instead of T.
// PRE2 (with PRE): res1 rows in pre, res2 rows in pre2 (both loaded by the caller ahead of its K
// loop, rows pix(i) of zero page when absent); bbias is still read here.
template <typename T, int TM, bool LN = false, bool PRE = false, bool Q8 = false, bool PRE2 = false, class PixOf>
DEV void epi_regs16(const ConvArgs& a, const f32x4 (&acc)[TM][4], const float (&bi)[16], int nb, int b,
                    const PixOf& pix, const EpiPref<TM>* pre = nullptr, const float* ssl = nullptr,
                    const EpiPref<TM>* pre2 = nullptr) {
  static_assert(!PRE2 || PRE, "PRE2 extends PRE");
  T* y = reinterpret_cast<T*>(a.y);
  __builtin_amdgcn_sched_barrier(0);             // (not hoisted into the MFMA phase)
  if constexpr (PRE) {
    // Every prefetched register stays allocated until here (after the caller's wait), also the
    // ones this epilogue does not read (TM < 4 duplicates): a register freed earlier could be
    // reused while its load is still in flight and then be overwritten when the load lands.
#pragma unroll
    for (int k = 0; k < (int)(sizeof(pre->v) / sizeof(pre->v[0])); ++k) asm volatile("" :: "v"(pre->v[k]));
  }
  if constexpr (PRE2) {
#pragma unroll
    for (int k = 0; k < (int)(sizeof(pre2->v) / sizeof(pre2->v[0])); ++k) asm volatile("" :: "v"(pre2->v[k]));
  }
  float sc[16], sh[16];
  if (a.ss && ssl) {                             // scale / shift rows staged in LDS by the caller
#pragma unroll
    for (int e = 0; e < 16; ++e) { sc[e] = ssl[e] + 1.f; sh[e] = ssl[64 + e]; }
  } else if (a.ss) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(a.ss + (size_t)b * a.ss_ld + nb);
    const u32x4* h4 = reinterpret_cast<const u32x4*>(a.ss + (size_t)b * a.ss_ld + a.Cout + nb);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 u, w;
      if constexpr (PRE) { u = pre->v[q]; w = pre->v[4 + q]; } else { u = s4[q]; w = h4[q]; }
#pragma unroll
      for (int e = 0; e < 4; ++e) { sc[4 * q + e] = __uint_as_float(u[e]) + 1.f; sh[4 * q + e] = __uint_as_float(w[e]); }
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) { sc[e] = 1.f; sh[e] = 0.f; }
  }
  float bb[16];
  if ((!PRE || PRE2) && a.bbias) {
#pragma unroll
    for (int e = 0; e < 16; ++e) bb[e] = a.bbias[(size_t)b * a.bb_ld + nb + e];
  }
  float gl[16];
  if constexpr (LN) {
#pragma unroll
    for (int e = 0; e < 16; ++e) gl[e] = a.ln_g[nb + e];
  }
  // Per channel, once per tile: the folded terms of conv_epi.h epi_fold (bias into the shift,
  // SiLU in the log2 domain: three VALU + v_exp + v_rcp per value instead of five + the two; the
  // epilogue's VALU is what the co-resident block's MFMAs must cover). The
  // activation is a uniform branch around the whole loop, not a per-value select.
  const bool silu = a.act == ACT_SILU;
#pragma unroll
  for (int e = 0; e < 16; ++e) epi_fold(bi[e], sc[e], sh[e], silu);
  auto body = [&](auto silu_c) {
  constexpr bool SILU = decltype(silu_c)::value;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const size_t m = pix(i);
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float u = fmaf(acc[i][e >> 2][e & 3], sc[e], sh[e]);
      v[e] = SILU ? silu_log2(u) : u;
    }
    if constexpr (LN) {
      float sm = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) sm += v[e];
      sm = red16_sum(sm);
      sm = red32_sum(sm);
      const float mean = sm * (1.f / 64.f);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) { const float d = v[e] - mean; q += d * d; }
      q = red16_sum(q);
      q = red32_sum(q);
      const float rstd = 1.f / sqrtf(q * (1.f / 64.f) + a.ln_eps);
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = (v[e] - mean) * rstd * gl[e];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (a.res1) {
        const u32x4 r1 = PRE ? pre->v[2 * i + h]
                             : *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(a.res1) + m * a.ldr1 + nb + 8 * h);
#pragma unroll
        for (int w = 0; w < 4; ++w) add_pair<T>(r1[w], v[8 * h + 2 * w], v[8 * h + 2 * w + 1]);
      }
      if ((!PRE || PRE2) && a.res2) {
        const u32x4 r2 = PRE2 ? pre2->v[2 * i + h]
                              : *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(a.res2) + m * a.ldr2 + nb + 8 * h);
#pragma unroll
        for (int w = 0; w < 4; ++w) add_pair<T>(r2[w], v[8 * h + 2 * w], v[8 * h + 2 * w + 1]);
      }
      if ((!PRE || PRE2) && a.bbias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[8 * h + e] += bb[8 * h + e];
      }
      if constexpr (!Q8) store_vec<T>(y + m * a.ldy + nb + 8 * h, v + 8 * h);
    }
    if constexpr (Q8) q8_store(a, m, nb, v);
  }
  };
  if (silu) body(std::true_type{});
  else body(std::false_type{});
}

// ---------------------------------------------------------------------------------------
// v2: NW = WGM*WGN waves, STAGES-deep LDS ring filled by global_load_lds (LDS-DMA, 16 B per
// lane, no register staging). Padding rows / K tail read a 16-byte zero page. The LDS image
// is lane-linear per wave-instruction (8 rows x 128 B), so the (row>>1)&7 slot swizzle is
// applied on the SOURCE address: lane l fills physical slot l&7 with logical slot
// (l&7) ^ ((row>>1)&7). Per K tile: wait own DMA of tile kt (counted vmcnt), barrier, refill
// the slot read in the previous iteration with tile kt+STAGES-1, then MFMA on tile kt.
// Requires Cin % (128/sizeof(T)) == 0 so a K tile covers one (kh, kw) tap.
typedef __attribute__((address_space(3))) void lds_void_t;
// One 16-byte-per-lane LDS-DMA through a raw buffer descriptor (base, nbytes): voff is the
// lane's byte offset, soff a wave-uniform one; an offset past nbytes lands zeros in LDS.
DEV void buf_lds16(const void* base, int nbytes, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes, 0x00020000), (lds_void_t*)lds, 16,
      voff, soff, 0, 0);
}
typedef __attribute__((address_space(1))) const void gbl_void_t;

template <typename T, int BM, int BN, int WGM, int WGN, int STAGES, int KH, int KW, int S, int P,
          int EPK = EPI_ALL>
__global__ void __launch_bounds__(64 * WGM * WGN) conv2_kernel(ConvArgs a) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int NW = WGM * WGN;
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int BKE = 128 / sizeof(T);
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int AG = BM / (8 * NW), BG = BN / (8 * NW);
  constexpr int KSTEPS = BKE / Mma<T>::KSTEP;
  constexpr int STAGE = (BM + BN) * 128;
  static_assert(AG >= 1 && BG >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile");
  // EPI_LNF (1x1 only): the input row LayerNorm folded in (ConvArgs::lnf_cs); EPE = the rest.
  constexpr bool LNF = (EPK & EPI_LNF) != 0;
  // EPI_GNA (1x1, swapped tiles): input GroupNorm applied to the A fragments from a per-channel
  // (scale, shift) table of this block's image, built in LDS behind the pipeline.
  constexpr bool GNA = (EPK & EPI_GNA) != 0;
  constexpr bool PART = (EPK & EPI_PART) != 0;
  constexpr int EPE = EPK & ~(EPI_LNF | EPI_GNA | EPI_PART);
  static_assert(!PART || (!LNF && !GNA && KH == 1 && KW == 1), "split-K: plain 1x1 GEMMs");
  static_assert(!LNF || (KH == 1 && KW == 1 && sizeof(T) == 2 && (EPK & EPI_SWAP)), "LN fold: 16-bit 1x1 swapped GEMMs");
  static_assert(!GNA || (KH == 1 && KW == 1 && sizeof(T) == 2 && (EPE & EPI_SWAP) && !LNF), "GN in A: 16-bit 1x1 swapped");
  constexpr bool SWAP = (EPE & EPI_SWAP) != 0;
  constexpr bool SLN = (EPE & EPI_LN) != 0 && SWAP;
  // EPI_SWAP | EPI_GEGLU: weights in the swapped GEGLU order (ConvArgs::w_gs), register epilogue.
  constexpr bool SGEGLU = EPE == (EPI_SWAP | EPI_GEGLU);
  static_assert(!SWAP || ((EPE == EPI_SWAP || SGEGLU || (EPE == (EPI_SWAP | EPI_LN) && WGN == 1 && BN == 64)) &&
                          TN == 4 && sizeof(T) == 2), "swapped tiles");
  constexpr int PIPE = STAGES * STAGE;
  constexpr int EPR = epi_rows<BM, BN, WTM>(PIPE);
  // (scale, shift) x Cin <= 512, (mean, rstd) x 64 groups: 4.5 KB, so three 64x128 blocks still
  // share a CU (3 x 53.75 KB).
  constexpr int GTAB = GNA ? 4096 + 512 : 0;
  constexpr int SMEM = (PIPE > EpiLds<EPR, BN>::BYTES ? PIPE : EpiLds<EPR, BN>::BYTES) + GTAB;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int HWo = a.Ho * a.Wo;
#ifdef DAC_STAMP
  // Diagnostic build only (tools/convbench_stamp): per-block shader-clock stamps into a.part.
  unsigned long long* stp = (!PART && a.part)
      ? reinterpret_cast<unsigned long long*>(a.part) + (size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8
      : nullptr;
#define DAC_ST(i, v) do { if (stp && tid == 0) stp[i] = (v); } while (0)
#else
#define DAC_ST(i, v) do { } while (0)
#endif
  DAC_ST(0, __builtin_amdgcn_s_memtime());
  DAC_ST(1, __builtin_amdgcn_s_memrealtime());
  kernarg_touch<sizeof(ConvArgs)>();
  DAC_ST(7, __builtin_amdgcn_s_memtime());
  const TileId tl = xcd_tile();
  const bool batched = a.w_bstride > 0;
  const int M = batched ? (tl.bz + 1) * HWo : a.B * HWo;
  const int m0 = (batched ? tl.bz * HWo : 0) + tl.bx * BM, n0 = tl.by * BN;
  float* gtab = reinterpret_cast<float*>(smem + (SMEM - GTAB));
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  const T* wgt = reinterpret_cast<const T*>(a.w) + (batched ? tl.bz * a.w_bstride : 0);

  // This lane's rows: A row (wave*AG + j)*8 + lane/8, B row (wave*BG + j)*8 + lane/8.
  int a_pix[AG], a_ih[AG], a_iw[AG], a_ls[AG], a_m[AG];
#pragma unroll
  for (int j = 0; j < AG; ++j) {
    const int row = (wave * AG + j) * 8 + (lane >> 3);
    a_ls[j] = (lane & 7) ^ ((row >> 1) & 7);
    const int m = m0 + row;
    a_m[j] = m;
    if (m < M) {
      if constexpr (KH == 1 && KW == 1 && S == 1 && P == 0) {
        // Pointwise: row m reads pixel m; only its validity is needed (no divisions: the
        // prologue's integer divisions were ~0.5 us of a 9 us GEMM, tools/convbench_stamp).
        a_pix[j] = 0; a_ih[j] = 0; a_iw[j] = 0;
      } else {
        const int b = m / HWo, r = m - b * HWo;
        const int oh = r / a.Wo, ow = r - oh * a.Wo;
        a_pix[j] = b * a.Hs * a.Ws;
        a_ih[j] = oh * S - P;
        a_iw[j] = ow * S - P;
      }
    } else {
      a_pix[j] = 0; a_ih[j] = -100000; a_iw[j] = -100000;
    }
  }
  const T* b_row[BG];
  int b_ls[BG];
#pragma unroll
  for (int j = 0; j < BG; ++j) {
    const int row = (wave * BG + j) * 8 + (lane >> 3);
    b_ls[j] = (lane & 7) ^ ((row >> 1) & 7);
    const int n = n0 + (SWAP ? (row & ~63) + wperm64(row & 63) : row);
    b_row[j] = n < a.Cout ? wgt + (size_t)n * a.K : nullptr;
  }
  // K tiles of this block: all, or split z's contiguous share (EPI_PART, grid z = ksplit).
  const int nk_all = (a.K + BKE - 1) / BKE;
  const int kt0 = PART ? (int)((long)tl.bz * nk_all / gridDim.z) : 0;
  const int nk = PART ? (int)((long)(tl.bz + 1) * nk_all / gridDim.z) - kt0 : nk_all;
  // 1x1 with ConvArgs::dbuf: buffer-descriptor DMA. Per-lane byte offsets (pixel row x pitch +
  // slot; weight row x K + slot) computed once, the K advance in the scalar soffset, rows past
  // M / Cout (and K tiles past K) as out-of-range offsets that land zeros -- no 64-bit address
  // arithmetic per DMA instruction.
  constexpr unsigned OOB = 0x80000000u;
  constexpr bool DB1 = KH == 1 && KW == 1 && S == 1 && P == 0;
  int a_bo[DB1 ? AG : 1], b_bo[DB1 ? BG : 1];
  int x1_bytes = 0, x2_bytes = 0, w_bytes = 0;
  if constexpr (DB1) {
    if (a.dbuf) {
      x1_bytes = a.B * a.Hs * a.Ws * a.ld1 * (int)sizeof(T);
      x2_bytes = a.x2 ? a.B * a.Hs * a.Ws * a.ld2 * (int)sizeof(T) : 0;
      w_bytes = a.Cout * a.K * (int)sizeof(T);
#pragma unroll
      for (int j = 0; j < AG; ++j) a_bo[j] = a_ih[j] >= 0 ? (a_m[j] * a.ld1 + a_ls[j] * VE) * (int)sizeof(T) : (int)OOB;
#pragma unroll
      for (int j = 0; j < BG; ++j) {
        const int row = (wave * BG + j) * 8 + (lane >> 3);
        const int n = n0 + (SWAP ? (row & ~63) + wperm64(row & 63) : row);
        b_bo[j] = n < a.Cout ? (n * a.K + b_ls[j] * VE) * (int)sizeof(T) : (int)OOB;
      }
    }
  }

  auto issue = [&](int kt) {
    char* st = smem + (kt % STAGES) * STAGE;
    const int k0 = (kt0 + kt) * BKE;
    const bool kv = kt < nk && k0 < a.K;
    if constexpr (KH == 7 && sizeof(T) == 2) {
      // Row-tap layout (kernel row padded to 8 taps, Cin = 8 = one 16-byte vector): K tile kt
      // is kernel row kh = kt, and logical slot s of a pixel row is tap kw = s (s = 7: zero).
      // Split-precision weights (cwrap): K tiles KH..2KH-1 are the lo rows of kernel rows 0..KH-1.
      const int kr = (a.cwrap && kt >= KH) ? kt - KH : kt;
#pragma unroll
      for (int j = 0; j < AG; ++j) {
        const int kw = a_ls[j];
        const int ih = a_ih[j] + kr, iw = a_iw[j] + kw;
        const char* src = zero;
        if (kv && kw < KW && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win)
          src = reinterpret_cast<const char*>(x1 + (size_t)(a_pix[j] + ih * a.Ws + iw) * a.ld1);
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + (wave * AG + j) * 8 * 128), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < BG; ++j) {
        const char* src = zero;
        if (kv && b_row[j]) src = reinterpret_cast<const char*>(b_row[j] + k0 + b_ls[j] * VE);
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + BM * 128 + (wave * BG + j) * 8 * 128),
                                         16, 0, 0);
      }
      return;
    }
    if constexpr (KH == 1 && KW == 1 && S == 1 && P == 0) {
      // Pointwise conv / linear (never upsampled, K = Cin): row m reads pixel m.
      int ci0 = k0;
      if (a.cwrap && ci0 >= a.cwrap) ci0 -= a.cwrap;
      const bool from1 = ci0 < a.C1;
      if (a.dbuf) {
        const int soa = (from1 ? ci0 : ci0 - a.C1) * (int)sizeof(T), sob = k0 * (int)sizeof(T);
#pragma unroll
        for (int j = 0; j < AG; ++j)
          buf_lds16(from1 ? a.x1 : a.x2, from1 ? x1_bytes : x2_bytes, st + (wave * AG + j) * 8 * 128,
                    kv ? a_bo[j] : (int)OOB, soa);
#pragma unroll
        for (int j = 0; j < BG; ++j)
          buf_lds16(wgt, w_bytes, st + BM * 128 + (wave * BG + j) * 8 * 128, kv ? b_bo[j] : (int)OOB, sob);
        return;
      }
      const char* xs = from1 ? reinterpret_cast<const char*>(x1 + ci0) : reinterpret_cast<const char*>(x2 + (ci0 - a.C1));
      const size_t ldb = (size_t)(from1 ? a.ld1 : a.ld2) * sizeof(T);
#pragma unroll
      for (int j = 0; j < AG; ++j) {
        const char* src = (kv && a_ih[j] >= 0) ? xs + (size_t)a_m[j] * ldb + a_ls[j] * 16 : zero;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + (wave * AG + j) * 8 * 128), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < BG; ++j) {
        const char* src = zero;
        if (kv && b_row[j]) src = reinterpret_cast<const char*>(b_row[j] + k0 + b_ls[j] * VE);
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + BM * 128 + (wave * BG + j) * 8 * 128),
                                         16, 0, 0);
      }
      return;
    }
    const int kpos = k0 / a.Cin;                 // wave-uniform (Cin % BKE == 0)
    int ci0 = k0 - kpos * a.Cin;
    if (a.cwrap && ci0 >= a.cwrap) ci0 -= a.cwrap;   // split-precision weights (cwrap % BKE == 0)
    const int kh = kpos / KW, kw = kpos - (kpos / KW) * KW;
#pragma unroll
    for (int j = 0; j < AG; ++j) {
      const int ih = a_ih[j] + kh, iw = a_iw[j] + kw;
      const int ci = ci0 + a_ls[j] * VE;
      const char* src = zero;
      if (kv && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win) {
        const int sh = a.up ? (ih >> 1) : ih, sw = a.up ? (iw >> 1) : iw;
        const size_t pix = (size_t)(a_pix[j] + sh * a.Ws + sw);
        src = reinterpret_cast<const char*>(ci < a.C1 ? x1 + pix * a.ld1 + ci
                                                      : x2 + pix * a.ld2 + (ci - a.C1));
      }
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(st + (wave * AG + j) * 8 * 128), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BG; ++j) {
      const char* src = zero;
      if (kv && b_row[j]) src = reinterpret_cast<const char*>(b_row[j] + k0 + b_ls[j] * VE);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(st + BM * 128 + (wave * BG + j) * 8 * 128),
                                       16, 0, 0);
    }
  };
  auto swz = [](int row, int s) { return row * 128 + ((s ^ ((row >> 1) & 7)) << 4); };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LN fold: this lane's partial row sums (sum d, sum d^2, d = x - shift) of A rows
  // wm*WTM + i*16 + lr over the K slices it reads (8 of every 32); summed over the four lane
  // groups after the loop. The shift is the row's first element (read from the first K tile in
  // LDS by all four lane groups of the row), so a row whose mean is many standard deviations
  // from zero keeps its variance: the moments are taken about a point inside the row.
  float ls1[LNF ? TM : 1], ls2[LNF ? TM : 1], lsh[LNF ? TM : 1];
#pragma unroll
  for (int i = 0; i < (LNF ? TM : 1); ++i) ls1[i] = ls2[i] = lsh[i] = 0.f;

  DAC_ST(6, __builtin_amdgcn_s_memtime());
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(s);
  if constexpr (GNA) {
    // Channel c of this tile's image: s = rstd * gamma, t = beta - mean * s (tile in one image:
    // conv_gna_ok). Its loads overlap the first stage's DMA; read after the first barrier.
    const int bimg = m0 / HWo, cpg = a.Cin / a.gna_groups;
    const float* stt = a.gna_stats + (size_t)bimg * a.gna_groups * 2;
    if (a.gna_nb > 0) {
      // Per-block (sum, sum of squares) of the PreNorm LayerNorm: tpg threads per group sum a
      // strided share of the image's nb blocks, then a fixed xor tree (lanes of one wave).
      float* gst = gtab + 1024;
      const int tpg = 64 * NW / a.gna_groups, gi = tid / tpg, p = tid % tpg;
      const float* pp = a.gna_stats + (size_t)(bimg * a.gna_groups + gi) * a.gna_nb * 2;
      float s1 = 0.f, s2 = 0.f;
      for (int k = p; k < a.gna_nb; k += tpg) { s1 += pp[2 * k]; s2 += pp[2 * k + 1]; }
      for (int o = 1; o < tpg; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      if (p == 0) {
        const float n = (float)HWo * (float)cpg, mu = s1 / n, var = fmaxf(s2 / n - mu * mu, 0.f);
        gst[2 * gi] = mu;
        gst[2 * gi + 1] = 1.f / sqrtf(var + a.gna_eps);
      }
      __syncthreads();
      stt = gst;
    }
    for (int c = tid; c < a.Cin; c += 64 * NW) {
      const float* st = stt + (c / cpg) * 2;
      const float sc = st[1] * a.gna_g[c];
      gtab[2 * c] = sc;
      gtab[2 * c + 1] = a.gna_b[c] - st[0] * sc;
    }
  }
  const int lr = lane & 15, lg = lane >> 4;
  // Swapped tiles: the epilogue's residual rows (res1, res2) are requested here, ahead of the K
  // loop, by inline-asm loads the compiler's wait insertion cannot see; they land under the K
  // loop instead of after it (the block's epilogue was 2.4 us warm / 5 us cold of a 9-15 us
  // 512 -> 512 GEMM, tools/convbench_stamp). The loop's trailing vmcnt(0) covers them.
  constexpr bool RPF = SWAP && !PART && !LNF && !GNA && !SGEGLU;
  EpiPref<TM> rp1, rp2;
  const bool rpf = RPF && (a.res1 || a.res2) && !a.ss;
  if constexpr (RPF) {
    if (rpf) {
      const int nbr = n0 + wn * WTN + 16 * lg;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(rp1.v) / sizeof(rp1.v[0])); ++k) {
        const int i = k / 2 < TM ? k / 2 : TM - 1, h = k & 1;
        const size_t m = (size_t)m0 + wm * WTM + i * 16 + lr;
        ld_asm(rp1.v[k], a.res1 ? (const void*)(reinterpret_cast<const T*>(a.res1) + m * a.ldr1 + nbr + 8 * h) : a.zero);
        ld_asm(rp2.v[k], a.res2 ? (const void*)(reinterpret_cast<const T*>(a.res2) + m * a.ldr2 + nbr + 8 * h) : a.zero);
      }
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 1) {
      // Single buffer (K fits one tile, or LDS kept small for occupancy): fill, wait, use.
      if (kt > 0) __syncthreads();               // everyone is done reading the buffer
      issue(kt);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      // Own DMA of tile kt done (STAGES-2 younger tiles may stay in flight), then barrier.
      if constexpr (STAGES == 2) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else if constexpr (STAGES == 3) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(AG + BG) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"((STAGES - 2) * (AG + BG)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(kt + STAGES - 1);                    // refills the slot read at iteration kt-1
    }
    if (kt == 0) DAC_ST(2, __builtin_amdgcn_s_memtime());
    const char* A = smem + (kt % STAGES) * STAGE;
    const char* Bs = A + BM * 128;
    if constexpr (!GNA && !LNF && !SGEGLU && !(EPK & EPI_GEGLU) && !(BM == 256 && BN == 256) && STAGES > 1 && KSTEPS > 1) {
      // Plain GEMMs: both k-steps' fragments are read into separate register sets before the
      // tile's MFMAs, so a tile waits out one LDS latency instead of one per k-step (1 wave per
      // SIMD in the 4-wave tiles: nothing else hides it). Same MFMAs in the same order:
      // bit-identical. (The 256 x 256 tiles have no VGPRs to spare; the single-buffer K <= 64
      // tiles measured slower with it, fewer blocks per CU.)
      u32x4 pa[2][TM], pb[2][TN];
      auto ld = [&](int ks, int h) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          pa[h][i] = *reinterpret_cast<const u32x4*>(A + swz(wm * WTM + i * 16 + lr, ks * 4 + lg));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          pb[h][j] = *reinterpret_cast<const u32x4*>(Bs + swz(wn * WTN + j * 16 + lr, ks * 4 + lg));
      };
      ld(0, 0);
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        if (ks + 1 < KSTEPS) ld(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (SWAP) Mma<T>::run(acc[i][j], pb[ks & 1][j], pa[ks & 1][i]);
            else Mma<T>::run(acc[i][j], pa[ks & 1][i], pb[ks & 1][j]);
          }
      }
      continue;
    }
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      u32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const u32x4*>(A + swz(wm * WTM + i * 16 + lr, ks * 4 + lg));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const u32x4*>(Bs + swz(wn * WTN + j * 16 + lr, ks * 4 + lg));
      if constexpr (GNA) {
        // This lane's 8 channels kt*BKE + ks*32 + lg*8 .. +7 (K = Cin for a 1x1 conv).
        const f32x4* tp = reinterpret_cast<const f32x4*>(gtab + 2 * (kt * BKE + ks * 32 + lg * 8));
        const f32x4 t0 = tp[0], t1 = tp[1], t2 = tp[2], t3 = tp[3];
        const float sc[8] = {t0[0], t0[2], t1[0], t1[2], t2[0], t2[2], t3[0], t3[2]};
        const float sh[8] = {t0[1], t0[3], t1[1], t1[3], t2[1], t2[3], t3[1], t3[3]};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          typename Vec8<T>::t v;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            float lo, hi;
            unpack2<T>(fa[i][w], lo, hi);
            v[2 * w] = (T)fmaf(lo, sc[2 * w], sh[2 * w]);
            v[2 * w + 1] = (T)fmaf(hi, sc[2 * w + 1], sh[2 * w + 1]);
          }
          fa[i] = __builtin_bit_cast(u32x4, v);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (SWAP) Mma<T>::run(acc[i][j], fb[j], fa[i]);
          else Mma<T>::run(acc[i][j], fa[i], fb[j]);
        }
      if constexpr (LNF) {
        if (ks == 0 && kt == 0) {
          // Element 0 of row wm*WTM + i*16 + lr (logical slot 0), read by all four lane groups.
#pragma unroll
          for (int i = 0; i < TM; ++i) lsh[i] = to_f(*reinterpret_cast<const T*>(A + swz(wm * WTM + i * 16 + lr, 0)));
        }
        // The WGN waves of a row band read the same A fragments: each takes the moments of its
        // share of the k-steps (ks % WGN == wn; 8 VALU per fragment word made this loop VALU-bound
        // at 2x its MFMA time) and the shares are summed after the loop.
        if (WGN > 1 && ks % WGN != __builtin_amdgcn_readfirstlane(wn)) continue;   // (wave-uniform)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            float lo, hi;
            unpack2<T>(fa[i][w], lo, hi);
            lo -= lsh[i];
            hi -= lsh[i];
            ls1[i] += lo + hi;
            ls2[i] = fmaf(lo, lo, fmaf(hi, hi, ls2[i]));
          }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  DAC_ST(3, __builtin_amdgcn_s_memtime());
  if constexpr (LNF) {
    if constexpr (WGN > 1) {
      // Sum the WGN waves' k-step shares per lane, in wave order (every wave of the band forms the
      // same sums), through LDS: the K loop's reads are done after this barrier.
      static_assert(WGN * 2 * TM * 64 * 4 * WGM <= STAGES * STAGE, "LN-fold exchange fits the pipeline LDS");
      float* xm = reinterpret_cast<float*>(smem);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        xm[((wave * TM + i) * 2) * 64 + lane] = ls1[i];
        xm[((wave * TM + i) * 2 + 1) * 64 + lane] = ls2[i];
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int v = 0; v < WGN; ++v) {
          const int w = wm * WGN + v;
          s1 += xm[((w * TM + i) * 2) * 64 + lane];
          s2 += xm[((w * TM + i) * 2 + 1) * 64 + lane];
        }
        ls1[i] = s1;
        ls2[i] = s2;
      }
    }
    // Row moments -> acc = rstd * (acc - mean * cs[n]), the LN'd-input GEMM before its bias.
    const float inv_n = 1.f / (float)a.lnf_n;
    float mu[TM], rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float t1 = red32_sum(red16_sum(ls1[i])), t2 = red32_sum(red16_sum(ls2[i]));
      const float d = t1 * inv_n;                // mean of x - shift
      mu[i] = lsh[i] + d;
      rs[i] = 1.f / sqrtf(fmaxf(t2 * inv_n - d * d, 0.f) + a.lnf_eps);
    }
    {
      // Lane (lr, lg): pixel row i*16 + lr, channels nb .. nb+15 (acc[i][e >> 2][e & 3]).
      const int nb = n0 + wn * WTN + 16 * lg;
      float cs[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) cs[e] = a.lnf_cs[nb + e];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e >> 2][e & 3] = rs[i] * fmaf(-mu[i], cs[e], acc[i][e >> 2][e & 3]);
    }
  }
  if constexpr (PART) {
    // Raw partial sums: tile i row 4 lg + r is pixel m, column lr of tile j is channel n.
    float* pz = a.part + (size_t)tl.bz * M * a.Cout;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + 4 * lg + r, n = n0 + wn * WTN + j * 16 + lr;
          if (m < M && n < a.Cout) pz[(size_t)m * a.Cout + n] = acc[i][j][r];
        }
    return;
  }
  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;
  const int bimg = (m0 / HWo == mlast / HWo) ? m0 / HWo : -1;
  if constexpr (SGEGLU) {
    // Lane (lr, lg), pixel row i: x of output channels ob .. ob + 7 in acc elements 0..7, their
    // gate in 8..15 (w_gs order); (x + bx) * gelu(gate + bg), the LDS epilogue's formula, stored
    // as 16 bytes. The dispatcher guarantees whole tiles inside one image and Cout % BN == 0.
    const int nb = n0 + wn * WTN + 16 * lg, ob = nb / 2;
    float bi[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bi[e] = a.bias ? a.bias[nb + e] : 0.f;
    T* y = reinterpret_cast<T*>(a.y);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const size_t m = (size_t)m0 + wm * WTM + i * 16 + lr;
      float o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c)
        o[c] = (acc[i][c >> 2][c & 3] + bi[c]) * gelu_fast(acc[i][(8 + c) >> 2][(8 + c) & 3] + bi[8 + c]);
      store_vec<T>(y + m * a.ldy + ob, o);
    }
  } else if constexpr (SWAP) {
    // The dispatcher guarantees whole tiles inside one image and Cout % BN == 0.
    const int nb = n0 + wn * WTN + 16 * lg;
    float bi[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bi[e] = a.bias ? a.bias[nb + e] : 0.f;
    if constexpr (RPF && !SLN) {
      if (rpf) {
        epi_regs16<T, TM, false, true, false, true>(a, acc, bi, nb, bimg, [&](int i) { return (size_t)m0 + wm * WTM + i * 16 + lr; },
                                                    &rp1, nullptr, &rp2);
      } else {
        epi_regs16<T, TM, SLN>(a, acc, bi, nb, bimg, [&](int i) { return (size_t)m0 + wm * WTM + i * 16 + lr; });
      }
    } else {
      epi_regs16<T, TM, SLN>(a, acc, bi, nb, bimg, [&](int i) { return (size_t)m0 + wm * WTM + i * 16 + lr; });
    }
  } else {
    conv_epilogue_lds<T, BM, BN, WGM, WGN, EPR, EPE>(a, acc, smem, M, LinearRows{m0}, n0, HWo, bimg);
  }
#ifdef DAC_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DAC_ST(4, __builtin_amdgcn_s_memtime());
  DAC_ST(5, __builtin_amdgcn_s_memrealtime());
#undef DAC_ST
}


// ---------------------------------------------------------------------------------------
// v3 (3x3, stride 1, pad 1): row-halo tiles. A block owns BM output pixels laid out as
// RH image rows x RW columns (RW = min(Wo, 256), power of two >= 16). The K loop walks
// (Cin chunk of 128 B, kh): each stage holds the RH input rows (ih = oh + kh - 1) over
// RW + 2 columns once, and the three kw taps read shifted windows of it, so every input
// pixel of a row band is fetched once per kh instead of once per tap (im2col x3 -> x1).
// The stage also holds the 3 (kw) weight tiles. Two LDS stages, LDS-DMA fill.
// Row width of a v3 tile of BM pixels for this output, or 0 if the shape does not tile.
inline int conv3_rw(const ConvArgs& a, int BM = 256) {
  const int Wo = a.Wo, Ho = a.Ho;
  if (Wo <= 0 || (Wo & (Wo - 1))) {
    if (Wo % BM == 0) return BM;
    return 0;
  }
  const int RW = Wo < BM ? Wo : BM;
  if (RW < 16) return 0;
  const int RH = BM / RW;
  if (Ho % RH) return 0;
  return RW;
}

// CK = bytes of one LDS row (one K chunk of one pixel): 128 (8 slots) or 64 (4 slots). A
// wave-instruction of global_load_lds fills 64 / SLOTS rows; slot swizzle sl ^ f(row). An A
// fragment's 16 rows start at any row (the kw tap shifts them by 0..2 and output rows start at
// oy * (RW + 2)), so f must keep every ds_read_b128 lane group ({0-3,12-15,20-27}, ...) on
// distinct bank quads for odd starts too: f = row & 7 (8 slots) and ((row >> 2) & 1) * 2 (4 slots)
// do, found by enumerating the lane groups over every start (the earlier (row >> 1) & 7 was
// 2-way on odd starts: SQ_LDS_BANK_CONFLICT 17.8% of LDS cycles on the 512-channel 32² conv).
// BUF: buffer-descriptor DMA (as v4 FL bit 10): per-lane 32-bit offsets computed once, the chunk
// and kh advance in the scalar soffset, padding as out-of-range offsets -- no 64-bit address
// arithmetic per DMA instruction (v3 spent ~3 VALU per MFMA there). One row pitch required.
template <typename T, int BM, int BN, int WGM, int WGN, int CK, bool BUF = false>
__global__ void __launch_bounds__(64 * WGM * WGN) conv3_kernel(ConvArgs a, int RW) {
  kernarg_touch<sizeof(ConvArgs) + 4>();                     // every kernarg line once, one wait (common.h)
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int NW = WGM * WGN;
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int ES = sizeof(T);
  constexpr int BKE = CK / ES;
  constexpr int SLOTS = CK / 16, RPI = 64 / SLOTS;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int NPIX_MAX = BM + 2 * (BM / 16);           // RH * (RW + 2) with RW >= 16
  constexpr int AG = (NPIX_MAX + RPI * NW - 1) / (RPI * NW);
  constexpr int BG = 3 * BN / (RPI * NW);
  constexpr int AROWS = AG * RPI * NW;
  constexpr int STAGE = (AROWS + 3 * BN) * CK;
  constexpr int KSTEPS = BKE / Mma<T>::KSTEP;
  static_assert(SLOTS == 8 || SLOTS == 4, "CK");
  static_assert(BG >= 1 && (3 * BN) % (RPI * NW) == 0 && KSTEPS >= 1, "tile");
  constexpr int EPR = epi_rows<BM, BN, WTM>(2 * STAGE);
  constexpr int SMEM = 2 * STAGE > EpiLds<EPR, BN>::BYTES ? 2 * STAGE : EpiLds<EPR, BN>::BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int HWo = a.Ho * a.Wo;
  const int rws = __builtin_ctz(RW);                      // RW is a power of two
  const int RH = BM >> rws, RWP = RW + 2, NPIX = RH * RWP;
  const TileId tl = xcd_tile();
  const int tiles_w = a.Wo >> rws;
  const int tiles_img = (a.Ho / RH) * tiles_w;
  const int b = tl.bx / tiles_img;
  const int tr = tl.bx - b * tiles_img;
  const int oh0 = (tr / tiles_w) * RH, ow0 = (tr % tiles_w) << rws;
  const int n0 = tl.by * BN;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const int pixb = b * a.Hs * a.Ws;
  auto fsw = [](int row) { return SLOTS == 8 ? row & 7 : ((row >> 2) & 1) << 1; };

  // Per lane and A row j: source pixel index for each kh (-1 = padding) and the 16-byte slot
  // it fills (source-side swizzle).
  int a_pix[AG][3], a_ls[AG];
#pragma unroll
  for (int j = 0; j < AG; ++j) {
    const int p = (wave * AG + j) * RPI + lane / SLOTS;
    a_ls[j] = ((lane % SLOTS) ^ fsw(p)) * VE;
    const int oy = p / RWP, iw = ow0 + (p - oy * RWP) - 1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh0 + oy + kh - 1;
      int pix = -1;
      if (p < NPIX && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win)
        pix = pixb + (a.up ? (ih >> 1) : ih) * a.Ws + (a.up ? (iw >> 1) : iw);
      a_pix[j][kh] = pix;
    }
  }
  // B rows: weight row pointer (tap kw folded in) and slot.
  const T* b_ptr[BG];
  int b_ls[BG];
#pragma unroll
  for (int j = 0; j < BG; ++j) {
    const int row = (wave * BG + j) * RPI + lane / SLOTS;
    b_ls[j] = ((lane % SLOTS) ^ fsw(row)) * VE;
    const int n = n0 + row % BN;
    b_ptr[j] = n < a.Cout ? reinterpret_cast<const T*>(a.w) + (size_t)n * a.K + (row / BN) * a.Cin
                          : nullptr;
  }
  // LDS byte offsets of this lane's MFMA fragments (stage-relative).
  const int lr = lane & 15, lg = lane >> 4;
  auto swz = [&](int row, int sl) { return row * CK + ((sl ^ fsw(row)) << 4); };
  int aoff[TM][3][KSTEPS], boff[3][TN][KSTEPS];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WTM + i * 16 + lr;
    const int oy = r >> rws;
    const int p = oy * RWP + (r - (oy << rws));
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) aoff[i][kw][ks] = swz(p + kw, ks * 4 + lg);
  }
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int jn = 0; jn < TN; ++jn)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
        boff[kw][jn][ks] = AROWS * CK + swz(kw * BN + wn * WTN + jn * 16 + lr, ks * 4 + lg);

  const int nchunk = a.Cin / BKE;
  constexpr unsigned OOB = 0x80000000u;
  int a_bo[BUF ? AG : 1][3], b_bo[BUF ? BG : 1];
  const int x_bytes = BUF ? a.B * a.Hs * a.Ws * a.ld1 * ES : 0;
  const int w_bytes = BUF ? a.Cout * a.K * ES : 0;
  if constexpr (BUF) {
#pragma unroll
    for (int j = 0; j < AG; ++j)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
        a_bo[j][kh] = a_pix[j][kh] >= 0 ? (a_pix[j][kh] * a.ld1 + a_ls[j]) * ES : (int)OOB;
#pragma unroll
    for (int j = 0; j < BG; ++j) {
      const int row = (wave * BG + j) * RPI + lane / SLOTS;
      const int n = n0 + row % BN;
      b_bo[j] = n < a.Cout ? (int)(((size_t)n * a.K + (row / BN) * a.Cin + b_ls[j]) * ES) : (int)OOB;
    }
  }
  auto issue = [&](int c, int kh, int buf) {
    char* st = smem + buf * STAGE;
    const int ci0 = c * BKE;
    const bool from1 = ci0 < a.C1;
    if constexpr (BUF) {
      const int soa = (from1 ? ci0 : ci0 - a.C1) * ES, sob = (kh * 3 * a.Cin + ci0) * ES;
#pragma unroll
      for (int j = 0; j < AG; ++j)
        buf_lds16(from1 ? a.x1 : a.x2, x_bytes, st + (wave * AG + j) * RPI * CK, a_bo[j][kh], soa);
#pragma unroll
      for (int j = 0; j < BG; ++j)
        buf_lds16(a.w, w_bytes, st + AROWS * CK + (wave * BG + j) * RPI * CK, b_bo[j], sob);
      return;
    }
    const char* xs = reinterpret_cast<const char*>(from1 ? a.x1 : a.x2) +
                     (size_t)(from1 ? ci0 : ci0 - a.C1) * ES;
    const size_t ldb = (size_t)(from1 ? a.ld1 : a.ld2) * ES;
#pragma unroll
    for (int j = 0; j < AG; ++j) {
      const int pix = a_pix[j][kh];
      const char* src = pix >= 0 ? xs + (size_t)pix * ldb + a_ls[j] * ES : zero;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(st + (wave * AG + j) * RPI * CK), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BG; ++j) {
      const char* src = b_ptr[j] ? reinterpret_cast<const char*>(b_ptr[j] + kh * 3 * a.Cin + ci0 + b_ls[j])
                                 : zero;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(st + AROWS * CK + (wave * BG + j) * RPI * CK),
                                       16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const EpiTerms<TN> et = epi_terms<TN>(a, n0, b, wn * WTN);   // latency hidden by the K loop

  // One stage: 3 KSTEPS fragment groups (kw, ks). Group g + 1's fragments are read into the other
  // register set before group g's MFMAs, so each group's LDS latency hides behind the previous
  // group's MFMAs (read-then-use inside a group left ~4 MFMAs between a read and its first use:
  // SQ_WAIT_INST_ANY 35 % of wave cycles at two waves per SIMD).
  auto compute = [&](int buf) {
    const char* st = smem + buf * STAGE;
    constexpr int NG = 3 * KSTEPS;
    u32x4 fa[2][TM], fb[2][TN];
    auto load = [&](int g, int h) __attribute__((always_inline)) {
      const int kw = g / KSTEPS, ks = g % KSTEPS;
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[h][i] = *reinterpret_cast<const u32x4*>(st + aoff[i][kw][ks]);
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) fb[h][jn] = *reinterpret_cast<const u32x4*>(st + boff[kw][jn][ks]);
    };
    load(0, 0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) load(g + 1, (g + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);           // keep the reads ahead of this group's MFMAs
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN; ++jn) Mma<T>::run(acc[i][jn], fa[g & 1][i], fb[g & 1][jn]);
    }
  };
  auto sync_stage = [&]() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // Split-K (ConvArgs::ksplit > 1, grid z = ksplit): this block sums the Cin chunks of split
  // tl.bz only and writes raw fp32 partials; conv_part_reduce adds the splits in order and
  // applies the epilogue. The split count comes from one image's shape (engine conv_call), so an
  // image's summation order never depends on the batch.
  const bool part = a.ksplit > 1;
  const int c_lo = part ? (int)((long)tl.bz * nchunk / a.ksplit) : 0;
  const int c_hi = part ? (int)((long)(tl.bz + 1) * nchunk / a.ksplit) : nchunk;
  // Stages s = 3c + kh alternate buffers; kh is unrolled so the A source table index is static.
  issue(c_lo, 0, 0);
  int buf = 0;
  for (int c = c_lo; c < c_hi; ++c) {
    sync_stage();
    issue(c, 1, buf ^ 1);
    compute(buf);
    buf ^= 1;
    sync_stage();
    issue(c, 2, buf ^ 1);
    compute(buf);
    buf ^= 1;
    sync_stage();
    if (c + 1 < c_hi) issue(c + 1, 0, buf ^ 1);
    compute(buf);
    buf ^= 1;
  }
  struct Rows {
    int base, rws, Wo;
    DEV int operator()(int t) const { return base + (t >> rws) * Wo + (t & ((1 << rws) - 1)); }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const Rows rm{b * HWo + oh0 * a.Wo + ow0, rws, a.Wo};
  if (part) {
    // Tile i row 4 lg + r is block pixel t (rm(t) in the image), column lr of tile jn is channel n.
    const size_t M = (size_t)a.B * HWo;
    float* pz = a.part + (size_t)tl.bz * M * a.Cout;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jn = 0; jn < TN; ++jn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = wm * WTM + i * 16 + 4 * lg + r, n = n0 + wn * WTN + jn * 16 + lr;
          if (n < a.Cout) pz[(size_t)rm(t) * a.Cout + n] = acc[i][jn][r];
        }
    return;
  }
  conv_epilogue_lds<T, BM, BN, WGM, WGN, EPR, EPI_MIN>(a, acc, smem, (b + 1) * HWo, rm, n0, HWo, b, &et);
}

// ---------------------------------------------------------------------------------------
// v4 (3x3, stride 1, pad 1): row-halo tiles with INTERLEAVED accumulator rows. A wave owns
// WTM = 16*TM consecutive output pixels of one image row; its accumulator tile i, row m is
// pixel m*TM + i. The kw tap of tile i then reads the same LDS rows as the kw=0 fragment of
// tile i+kw, so one K step needs only TM+2 distinct A fragments (F_s, lane m: halo pixel
// m*TM + s) instead of 3*TM: tile i, tap kw multiplies F_{i+kw}. That cuts the A share of the
// LDS reads by ~2x, which (with the 64x64 wave tiles) keeps the CU's 256 B/clk LDS port below
// the MFMA rate.
// LDS image of a stage: the halo rows (logical row R = oy*(RW+2) + ox) then the 3*BN weight
// rows. Bank mapping (ds_read_b128 lane groups {0-3,12-15,20-27}, ...): a fragment read
// touches rows R0 + TM*m, so A rows are permuted within aligned groups of 4 (CK=64) or 2
// (CK=128) rows, P(R) = (R & ~QM) | ((R + (R >> QS)) & QM), and their 16-byte slots XORed with
// (R >> FS). The (QS, FS) pairs were found by exhaustive search over every row offset to make
// each lane group hit 16 distinct 16-byte bank quads; weight rows are read contiguously and
// use the TM = 1 pair. LDS-DMA writes stay lane-linear: each lane inverts P to find the
// logical row it fills. ST-deep ring, counted vmcnt (conservative for waves with one extra
// A instruction), one barrier per stage.
template <int SLOTS, int TM> struct Swz;
template <> struct Swz<4, 1> { static constexpr int QS = 0, FS = 1; };
template <> struct Swz<4, 2> { static constexpr int QS = 2, FS = 0; };
template <> struct Swz<4, 4> { static constexpr int QS = 2, FS = 3; };
template <> struct Swz<4, 8> { static constexpr int QS = 3, FS = 4; };
template <> struct Swz<8, 1> { static constexpr int QS = 0, FS = 0; };
template <> struct Swz<8, 2> { static constexpr int QS = 1, FS = 1; };
template <> struct Swz<8, 4> { static constexpr int QS = 2, FS = 2; };
template <> struct Swz<8, 8> { static constexpr int QS = 3, FS = 3; };

template <int SLOTS, int TM> struct RowSwz {
  static constexpr int QM = SLOTS == 4 ? 3 : 1;
  static constexpr int QS = Swz<SLOTS, TM>::QS, FS = Swz<SLOTS, TM>::FS;
  static_assert(QS == 0 || (1 << QS) > QM, "P must keep the bits above QM");
  DEV static int phys(int R) { return QS == 0 ? R : (R & ~QM) | ((R + (R >> QS)) & QM); }
  DEV static int logical(int P) { return QS == 0 ? P : (P & ~QM) | ((P - (P >> QS)) & QM); }
  DEV static int slot(int R, int L) { return L ^ ((R >> FS) & (SLOTS - 1)); }
};

// FL bit 0: sched_barrier fences around each stage (MFMAs stay inside their stage, so the
// stage's DMA wait overlaps them instead of preceding them); bit 1: all B fragments of a stage
// are read up front.
template <typename T, int BM, int BN, int WGM, int WGN, int CK, int ST, int FL = 0, int EPK = EPI_MIN, int WPE = 2>
__global__ void __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
conv3i_kernel(ConvArgs a, int RW) {
  kernarg_touch<sizeof(ConvArgs) + 4>();                     // every kernarg line once, one wait (common.h)
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int NW = WGM * WGN;
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int ES = sizeof(T);
  constexpr int BKE = CK / ES;
  constexpr int SLOTS = CK / 16, RPI = 64 / SLOTS;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int NF = TM + 2;                                 // distinct A fragments per K step
  constexpr int KSTEPS = BKE / Mma<T>::KSTEP;
  constexpr int QM = SLOTS == 4 ? 3 : 1;
  // Halo rows: RH*(RW+2) <= BM + 2*BM/WTM (RW >= WTM), rounded to the permutation group.
  constexpr int NPIX_MAX = BM + 2 * (BM / WTM);
  constexpr int NA_MAX = ((NPIX_MAX + QM) / (QM + 1) * (QM + 1) + RPI - 1) / RPI;
  constexpr int NA_MIN = (BM + 2 + RPI - 1) / RPI;
  constexpr int AGX = (NA_MAX + NW - 1) / NW;                // A DMA instructions per wave (max)
  constexpr int AGN = NA_MIN / NW;                           // ... (min, for the vmcnt count)
  constexpr int AROWS = NA_MAX * RPI;
  // FL bit 14 (with 13): column-phase too — the waves of a tile each hold output columns of one
  // parity b, whose three kernel columns fold to two taps over the SOURCE columns like the rows:
  // (W.0, W.1+W.2 | W.0+W.1, W.2). The halo is then source pixels (RW/2 + 2 per row, no
  // duplicates) and a stage's weight rows are the 4 (b, tap) sets: w is [Cout][4 row sets][4][Cin].
  constexpr bool UPC = (FL & 16384) != 0;
  constexpr int NBR = UPC ? 4 : 3;                           // weight-row sets per stage
  constexpr int NTAP = UPC ? 2 : 3;                          // taps per wave per stage
  constexpr int NB = NBR * BN / RPI;                         // B DMA instructions per stage
  constexpr int BGX = (NB + NW - 1) / NW, BGN = NB / NW;     // per wave (max / min)
  // FL bit 4: fused 1x1 second output (ConvArgs::w2 / y2): the centre-tap A fragments of the
  // kh = 1 stages also multiply the w2 rows (hi and lo parts), staged after the 3*BN weight
  // rows, into a second accumulator set written by a plain register epilogue.
  constexpr bool RES = (FL & 16) != 0;
  constexpr int RROWS = RES ? 2 * BN : 0;
  constexpr int STAGE = (AROWS + NBR * BN + RROWS) * CK;
  static_assert(SLOTS == 8 || SLOTS == 4, "CK");
  static_assert((NBR * BN) % RPI == 0 && KSTEPS >= 1 && TM >= 1 && TN >= 1, "tile");
  static_assert(!UPC || ((FL & 8192) && (FL & 8) && !RES && WGN == 1 && WTM == 64), "column-phase tiles");
  static_assert(!RES || (ST == 2 && (FL & 8) && BN % RPI == 0), "fused res: swapped tiles, 2 stages");
  static_assert(STAGE % 256 == 0 && (AROWS * CK) % 256 == 0, "bank-line aligned regions");
  static_assert(ST == 2 || ST == 3 || ST == 4, "stages");
  constexpr int VMW = (ST - 2) * (AGN + BGN);
  static_assert(VMW < 64, "vmcnt");
  // FL bit 3: swapped MFMA operands (weights as A) + register epilogue (epi_regs16).
  constexpr bool SWAP = (FL & 8) != 0;
  static_assert(!SWAP || (WTN == 64 && sizeof(T) == 2 && EPK == EPI_MIN && (!RES || BN == 64)), "swapped tiles");
  // Whole-tile epilogue (one pass, residual prefetch) whenever its fp32 tile still leaves room
  // for two blocks per CU; otherwise passes that fit in the pipeline's LDS.
  constexpr int EPR = EpiLds<BM, BN>::BYTES <= 80 * 1024 ? BM : epi_rows<BM, BN, WTM>(ST * STAGE);
  // Swapped tiles: 1 KB after the ring holds the tile's per-image scale / shift rows and bias
  // (64 channels each), DMA'd with the first stage, read by the epilogue from LDS.
  constexpr int SMEM = (FL & 8) ? ST * STAGE + 1024
                       : (ST * STAGE > EpiLds<EPR, BN>::BYTES ? ST * STAGE : EpiLds<EPR, BN>::BYTES);
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  using SA = RowSwz<SLOTS, TM>;
  using SB = RowSwz<SLOTS, 1>;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform in an SGPR
  const int wm = wave / WGN, wn = wave % WGN;
  const int HWo = a.Ho * a.Wo;
  const int rws = __builtin_ctz(RW);                      // RW is a power of two, RW % WTM == 0
  const int RH = BM >> rws, RWP = UPC ? RW / 2 + 2 : RW + 2, NPIX = RH * RWP;
  const int NA = ((NPIX + QM) / (QM + 1) * (QM + 1) + RPI - 1) / RPI;
  const TileId tl = xcd_tile();
  const int tiles_w = a.Wo >> rws;
  const int tiles_img = (a.Ho / RH) * tiles_w;
  const int b = tl.bx / tiles_img;
  const int tr = tl.bx - b * tiles_img;
  // FL bit 13 (row-phase upsample conv, ConvArgs::uph): tile row index tri = 2g + a holds the
  // output rows 2 RH g + a + 2y (one parity a), stride 2 Wo; its kernel-row stages s2 = 0, 1 read
  // source rows as kernel rows kh = s2 + a of the plain conv and weight rows 2a + s2.
  constexpr bool UPH = (FL & 8192) != 0;
  const int tri = tr / tiles_w;
  const int ph = UPH ? (tri & 1) : 0;
  const int oh0 = UPH ? 2 * RH * (tri >> 1) + ph : tri * RH, ow0 = (tr % tiles_w) << rws;
  constexpr int KHN = UPH ? 2 : 3;                         // kernel-row stages per chunk
  const int n0 = tl.by * BN;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const int pixb = b * a.Hs * a.Ws;

  // FL bit 10: buffer-resource DMA (buffer_load ... lds). Every per-lane source offset is a
  // 32-bit table entry computed once; the chunk and kh advance ride in the scalar soffset,
  // and padding pixels / rows past Cout carry an out-of-range offset, which the range check
  // turns into zeros in LDS -- the main loop issues its DMA with no VALU address arithmetic.
  // Requires ld2 == ld1 when the input is split (conv3i_buf_ok on the host).
  constexpr bool BUF = (FL & 1024) != 0;
  constexpr unsigned OOB = 0x80000000u;
  // A DMA: instruction j of this wave fills physical rows (wave + j*NW)*RPI + lane/SLOTS.
  int a_pix[AGX][KHN], a_ls[AGX];
#pragma unroll
  for (int j = 0; j < AGX; ++j) {
    const int P = (wave + j * NW) * RPI + lane / SLOTS;
    const int R = SA::logical(P);
    a_ls[j] = SA::slot(R, lane % SLOTS) * VE;
    const int oy = R / RWP, iw = ow0 + (R - oy * RWP) - 1;
    const int sw = (ow0 >> 1) + (R - oy * RWP) - 1;             // UPC: source column
#pragma unroll
    for (int kh = 0; kh < KHN; ++kh) {
      const int ih = UPH ? oh0 + 2 * oy + kh + ph - 1 : oh0 + oy + kh - 1;
      int pix = -1;
      if (UPC) {
        if (R < NPIX && (unsigned)ih < (unsigned)Hin && (unsigned)sw < (unsigned)a.Ws)
          pix = pixb + (ih >> 1) * a.Ws + sw;
      } else if (R < NPIX && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win) {
        pix = pixb + (a.up ? (ih >> 1) : ih) * a.Ws + (a.up ? (iw >> 1) : iw);
      }
      if constexpr ((FL & 2048) != 0) pix = pix >= 0 ? (pix & 255) : pix;   // diagnostic: L2-resident A rows
      a_pix[j][kh] = BUF ? (pix >= 0 ? (pix * a.ld1 + a_ls[j]) * ES : (int)OOB) : pix;
    }
  }
  // B DMA: instruction j of this wave fills weight rows (wave + j*NW)*RPI + lane/SLOTS
  // (row = tap kw * BN + channel).
  const T* b_ptr[BGX];
  int b_ls[BGX];
#pragma unroll
  for (int j = 0; j < BGX; ++j) {
    const int row = (wave + j * NW) * RPI + lane / SLOTS;
    b_ls[j] = SB::slot(row, lane % SLOTS) * VE;
    const int n = n0 + (SWAP ? (row % BN & ~63) + wperm64(row % BN & 63) : row % BN);
    b_ptr[j] = n < a.Cout ? reinterpret_cast<const T*>(a.w) + (size_t)n * a.K + (row / BN) * a.Cin
                          : nullptr;
    if constexpr (BUF) b_ls[j] = n < a.Cout ? (int)(((size_t)n * a.K + (row / BN) * a.Cin + b_ls[j]) * ES) : (int)OOB;
  }
  // Res-weight DMA: instruction j of this wave fills rows 3*BN + (wave + j*NW)*RPI + lane/SLOTS
  // (part = local row / BN: 0 hi, 1 lo).
  constexpr int RGX = RES ? (RROWS / RPI + NW - 1) / NW : 1;
  const T* r_ptr[RGX];
  int r_ls[RGX];
  const int nparts = RES && a.w2_dual ? 2 : 1;
  if constexpr (RES) {
#pragma unroll
    for (int j = 0; j < RGX; ++j) {
      const int lrow = (wave + j * NW) * RPI + lane / SLOTS;
      const int row = NBR * BN + lrow;
      r_ls[j] = SB::slot(row, lane % SLOTS) * VE;
      const int part = lrow / BN;
      const int n = n0 + wperm64(lrow % BN);
      r_ptr[j] = (lrow < RROWS && part < nparts && n < a.Cout)
                     ? reinterpret_cast<const T*>(a.w2) + (size_t)n * a.Cin * nparts + part * a.Cin
                     : nullptr;
      if constexpr (BUF)
        r_ls[j] = r_ptr[j] ? (int)(((size_t)n * a.Cin * nparts + part * a.Cin + r_ls[j]) * ES) : (int)OOB;
    }
  }
  // Buffer sizes (bytes) for the range check; the descriptors are built at each DMA from
  // kernel-argument bases (wave-uniform by construction; the compiler hoists them).
  const int x_bytes = BUF ? a.B * a.Hs * a.Ws * a.ld1 * ES : 0;
  const int w_bytes = BUF ? a.Cout * a.K * ES : 0;
  const int w2_bytes = BUF && RES && a.w2 ? a.Cout * a.Cin * nparts * ES : 0;
  // Fragment offsets (stage-relative bytes).
  const int lr = lane & 15, lg = lane >> 4;
  int aoff[NF][KSTEPS], boff[NTAP][TN][KSTEPS];
  // UPC: wave wm = (row y, column parity cb, 64-column part jo) of the tile; its fragment base
  // is shifted by cb so that tap t2 of tile i reads F[i + t2].
  const int upr = UPC ? (RW / 2) / 64 : 1;                  // waves per (row, parity)
  const int cy = UPC ? wm / (2 * upr) : 0, cb = UPC ? (wm % (2 * upr)) / upr : 0;
  const int cjo = UPC ? (wm % upr) * 64 : 0;
  {
    const int t0 = wm * WTM;
    const int R0 = UPC ? cy * RWP + cjo + cb + TM * lr : (t0 >> rws) * RWP + (t0 & (RW - 1)) + TM * lr;
#pragma unroll
    for (int s = 0; s < NF; ++s)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
        aoff[s][ks] = SA::phys(R0 + s) * CK + (SA::slot(R0 + s, ks * 4 + lg) << 4);
  }
#pragma unroll
  for (int kw = 0; kw < NTAP; ++kw)
#pragma unroll
    for (int jn = 0; jn < TN; ++jn)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int row = (UPC ? 2 * cb + kw : kw) * BN + wn * WTN + jn * 16 + lr;
        boff[kw][jn][ks] = AROWS * CK + row * CK + (SB::slot(row, ks * 4 + lg) << 4);
      }

  // kh must be a compile-time index into a_pix (a dynamic index sends the table to scratch).
  auto issue = [&](int c, auto khc, int buf) {
    constexpr int kh = decltype(khc)::value;
    if constexpr ((FL & 32) != 0) return;                       // diagnostic: no DMA
    char* st = smem + buf * STAGE;
    const int ci0 = c * BKE;
    const bool from1 = ci0 < a.C1;
    if constexpr (BUF) {
      const int soa = (from1 ? ci0 : ci0 - a.C1) * ES;
#pragma unroll
      for (int j = 0; j < AGX; ++j)
        if (wave + j * NW < NA)                                  // wave-uniform
          buf_lds16(from1 ? a.x1 : a.x2, x_bytes, st + (wave + j * NW) * RPI * CK, a_pix[j][kh], soa);
      const int sob = ((UPH ? 2 * ph + kh : kh) * NBR * a.Cin + ci0) * ES;
#pragma unroll
      for (int j = 0; j < BGX; ++j)
        if (BGX == BGN || wave + j * NW < NB)                    // wave-uniform
          buf_lds16(a.w, w_bytes, st + AROWS * CK + (wave + j * NW) * RPI * CK, b_ls[j], sob);
      if constexpr (RES && kh == 1) {
#pragma unroll
        for (int j = 0; j < RGX; ++j)
          if ((wave + j * NW) * RPI < RROWS)                       // wave-uniform
            buf_lds16(a.w2, w2_bytes, st + (AROWS + NBR * BN) * CK + (wave + j * NW) * RPI * CK, r_ls[j], ci0 * ES);
      }
      return;
    }
    const char* xs = reinterpret_cast<const char*>(from1 ? a.x1 : a.x2) +
                     (size_t)(from1 ? ci0 : ci0 - a.C1) * ES;
    const size_t ldb = (size_t)(from1 ? a.ld1 : a.ld2) * ES;
#pragma unroll
    for (int j = 0; j < AGX; ++j) {
      if (wave + j * NW < NA) {                                  // wave-uniform
        const int pix = a_pix[j][kh];
        const char* src = pix >= 0 ? xs + (size_t)pix * ldb + a_ls[j] * ES : zero;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + (wave + j * NW) * RPI * CK), 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BGX; ++j) {
      if (BGX == BGN || wave + j * NW < NB) {                   // wave-uniform
        const char* src = b_ptr[j] ? reinterpret_cast<const char*>(b_ptr[j] + (UPH ? 2 * ph + kh : kh) * NBR * a.Cin + ci0 + b_ls[j])
                                   : zero;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                         (lds_void_t*)(st + AROWS * CK + (wave + j * NW) * RPI * CK),
                                         16, 0, 0);
      }
    }
    if constexpr (RES && kh == 1) {
#pragma unroll
      for (int j = 0; j < RGX; ++j) {
        if ((wave + j * NW) * RPI < RROWS) {                        // wave-uniform
          const char* src = r_ptr[j] ? reinterpret_cast<const char*>(r_ptr[j] + ci0 + r_ls[j]) : zero;
          __builtin_amdgcn_global_load_lds(
              (gbl_void_t*)src, (lds_void_t*)(st + (AROWS + NBR * BN) * CK + (wave + j * NW) * RPI * CK), 16, 0, 0);
        }
      }
    }
  };

  f32x4 acc[TM][TN];
  f32x4 accR[RES ? TM : 1][RES ? TN : 1];
  if constexpr (RES) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) accR[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  EpiTerms<SWAP ? 1 : TN> et;
  if constexpr (!SWAP) et = epi_terms<TN>(a, n0, b, wn * WTN);   // latency hidden by the K loop

  auto compute = [&](int buf, auto khc) {
    constexpr int kh = decltype(khc)::value;
    const char* st = smem + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      u32x4 fa[NF];
#pragma unroll
      for (int s = 0; s < NF; ++s) fa[s] = *reinterpret_cast<const u32x4*>(st + aoff[s][ks]);
      if constexpr (RES && kh == 1) {
        // Fused res_conv: centre tap (kw = 1) fragments F_{i+1} times the w2 rows.
        for (int pt = 0; pt < nparts; ++pt) {
          u32x4 fr[TN];
#pragma unroll
          for (int jn = 0; jn < TN; ++jn) {
            const int row = NBR * BN + pt * BN + wn * WTN + jn * 16 + lr;
            fr[jn] = *reinterpret_cast<const u32x4*>(st + AROWS * CK + row * CK + (SB::slot(row, ks * 4 + lg) << 4));
          }
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jn = 0; jn < TN; ++jn) Mma<T>::run(accR[i][jn], fr[jn], fa[i + 1]);
        }
      }
      if constexpr ((FL & 2) && !UPC) {
        u32x4 fb[3][TN];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int jn = 0; jn < TN; ++jn) fb[kw][jn] = *reinterpret_cast<const u32x4*>(st + boff[kw][jn][ks]);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jn = 0; jn < TN; ++jn) {
              if constexpr (SWAP) Mma<T>::run(acc[i][jn], fb[kw][jn], fa[i + kw]);
              else Mma<T>::run(acc[i][jn], fa[i + kw], fb[kw][jn]);
            }
        continue;
      }
      if constexpr (FL & 4) __builtin_amdgcn_s_setprio(1);   // MFMA phase ahead of the
#pragma unroll                                                  // other block's DMA issue
      for (int kw = 0; kw < NTAP; ++kw) {
        u32x4 fb[TN];
#pragma unroll
        for (int jn = 0; jn < TN; ++jn) fb[jn] = *reinterpret_cast<const u32x4*>(st + boff[kw][jn][ks]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int jn = 0; jn < TN; ++jn) {
            if constexpr ((FL & 64) != 0) acc[i][jn][0] += __uint_as_float(fb[jn][0] ^ fa[i + kw][0]);  // diagnostic: no MFMA
            else if constexpr (SWAP) Mma<T>::run(acc[i][jn], fb[jn], fa[i + kw]);
            else Mma<T>::run(acc[i][jn], fa[i + kw], fb[jn]);
          }
      }
      if constexpr (FL & 4) __builtin_amdgcn_s_setprio(0);
    }
  };

  // Stage s = 3*c + kh. The loop is unrolled over kh so every issue() has a static kh: the
  // stage issued at (c, kh) is s + ST - 1 = (c + (kh + ST - 1) / 3, (kh + ST - 1) % 3).
  static_assert(!UPH || (ST == 2 && !RES), "row-phase tiles: 2 stages, no fused res_conv");
  const int nchunk = a.Cin / BKE, S = KHN * nchunk;
  issue(0, std::integral_constant<int, 0>{}, 0);
  if constexpr (SWAP) {
    if (wave == 0) {                              // lanes 0-15 scale, 16-31 shift, 32-47 bias
      const int part = lane >> 4, l16 = lane & 15;
      const float* src = reinterpret_cast<const float*>(zero);
      if (part == 0 && a.ss) src = a.ss + (size_t)b * a.ss_ld + n0 + 4 * l16;
      else if (part == 1 && a.ss) src = a.ss + (size_t)b * a.ss_ld + a.Cout + n0 + 4 * l16;
      else if (part == 2 && a.bias) src = a.bias + n0 + 4 * l16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(smem + ST * STAGE), 16, 0, 0);
    }
  }
  if constexpr (ST >= 3) issue(0, std::integral_constant<int, 1>{}, 1);
  if constexpr (ST >= 4) issue(0, std::integral_constant<int, 2>{}, 2);
  int buf = 0, nbuf = ST - 1;
  // Swapped tiles without the fused res_conv: the epilogue's residual rows are loaded at the
  // start of the last stage (inline asm, so they stay there), landing under its MFMAs instead of
  // after them (the fused variant has no registers left for them).
  const bool pre_ok = SWAP && !RES && a.res1 && !a.res2 && !a.bbias && !a.ss;
  EpiPref<TM> pref;
  const int rm_base = b * HWo + oh0 * a.Wo + ow0;
  const int rstride = UPH ? 2 * a.Wo : a.Wo;              // output row stride of the tile
  // UPC: the wave's pixel t is output column ow0 + 2 (cjo + t) + cb of row oh0 + 2 cy.
  const int upc_base = b * HWo + (oh0 + 2 * cy) * a.Wo + ow0 + 2 * cjo + cb;
  auto pixf = [&](int i) {
    const int t = wm * WTM + TM * lr + i;
    if constexpr (UPC) return (size_t)(upc_base + 2 * (TM * lr + i));
    return (size_t)(rm_base + (t >> rws) * rstride + (t & ((1 << rws) - 1)));
  };
  auto step = [&](int c, auto khc) {
    constexpr int kh = decltype(khc)::value;
    constexpr int KN = (kh + ST - 1) % KHN, CN = (kh + ST - 1) / KHN;
    const int s = KHN * c + kh;
    if constexpr (FL & 1) __builtin_amdgcn_sched_barrier(0);
    if (s + ST - 2 < S) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(VMW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr ((FL & 256) == 0) __builtin_amdgcn_s_barrier();   // (FL 256: diagnostic, no barrier)
    asm volatile("" ::: "memory");
    if (s + ST - 1 < S) issue(c + CN, std::integral_constant<int, KN>{}, nbuf);
    if constexpr (SWAP && kh == KHN - 1) {
      if (s + 1 == S && pre_ok) {
        const int nb = n0 + wn * WTN + 16 * lg;
        epi_prefetch<T, TM>(a, nb, b, pixf, pref);
      }
    }
    if constexpr (FL & 1) __builtin_amdgcn_sched_barrier(0);
    compute(buf, khc);
    buf = buf + 1 == ST ? 0 : buf + 1;
    nbuf = nbuf + 1 == ST ? 0 : nbuf + 1;
  };
  for (int c = 0; c < nchunk; ++c) {
    step(c, std::integral_constant<int, 0>{});
    step(c, std::integral_constant<int, 1>{});
    if constexpr (!UPH) step(c, std::integral_constant<int, 2>{});
  }
  struct Rows {
    int base, rws, Wo;
    DEV int operator()(int t) const { return base + (t >> rws) * Wo + (t & ((1 << rws) - 1)); }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const Rows rm{b * HWo + oh0 * a.Wo + ow0, rws, rstride};
  if constexpr ((FL & 128) != 0) {                 // diagnostic: no epilogue (all MFMA chains kept live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1.2345e-30f) reinterpret_cast<float*>(a.y)[tid] = t;
    return;
  }
  if constexpr (SWAP) {
    const int nb = n0 + wn * WTN + 16 * lg;
    float bi[16];
    const float* el = reinterpret_cast<const float*>(smem + ST * STAGE) + 16 * lg;   // LDS terms
#pragma unroll
    for (int e = 0; e < 16; ++e) bi[e] = el[128 + e];
    // FL bit 12: fp8 output (ConvArgs::ys8, q8_store) — the fp8 handles' block1 with a fused
    // res_conv, whose y2 stays 16-bit.
    constexpr bool Q8 = (FL & 4096) != 0;
    if constexpr (UPC) {
      if (pre_ok) epi_regs16<T, TM, false, true, Q8>(a, acc, bi, nb, b, pixf, &pref, el);
      else epi_regs16<T, TM, false, false, Q8>(a, acc, bi, nb, b, pixf, nullptr, el);
    } else {
      if (pre_ok) epi_regs16<T, TM, false, true, Q8>(a, acc, bi, nb, b, [&](int i) { return (size_t)rm(wm * WTM + TM * lr + i); }, &pref, el);
      else epi_regs16<T, TM, false, false, Q8>(a, acc, bi, nb, b, [&](int i) { return (size_t)rm(wm * WTM + TM * lr + i); }, nullptr, el);
    }
    if constexpr (RES) {
      // y2 = accR (+ bias2): lane holds channels nb .. nb+15 of pixel rows i (as epi_regs16).
      T* y2 = reinterpret_cast<T*>(a.y2);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const size_t m = (size_t)rm(wm * WTM + TM * lr + i);
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = accR[i][e >> 2][e & 3] + (a.bias2 ? a.bias2[nb + e] : 0.f);
        store_vec<T>(y2 + m * a.ldy2 + nb, v);
        store_vec<T>(y2 + m * a.ldy2 + nb + 8, v + 8);
      }
    }
  } else {
    conv_epilogue_lds<T, BM, BN, WGM, WGN, EPR, EPK, TM>(a, acc, smem, (b + 1) * HWo, rm, n0, HWo, b, &et);
  }
}

// Conv3 kernel choice override for microbenchmarks (tools/convbench): -1 = built-in choice,
// 0 = v3 only, k > 0 = v4 configuration k of conv3i_launch.
extern int g_conv3_force;
extern int g_conv2_force;     // 1x1 v2 configuration override (convbench), 0 = built-in
extern int g_conv2_force32;   // the same, small images only (DAC_CONV2_FORCE32)
extern int g_conv3_buf;       // v4 buffer-resource DMA (FL bit 10); DAC_CONV3_BUF=0 disables
extern int g_conv3h_on;       // v6 2-D halo kernel: 0 off, 1 measured-faster shapes, 2 all (DAC_CONV3H)
// Ring depth of the plain v4 swapped tiles (no fused res_conv, no phase form) when the grid is at
// most one block per CU (the 64x64 / 32x32 levels at B = 8): with no co-resident block to cover a
// stage's DMA, deeper rings keep more of it in flight (DAC_C3I_ST = 2 / 3 / 4; 3 measured best: 32x32
// 256->256 21.6 -> 18.9 us, 64x64 128->128 18.2 -> 17.6 us in the network, +0.45 % images/s). The stage count only
// buffers: every output is the same ordered sum, so the choice leaves results bit-identical.
extern int g_c3i_st;
extern int g_geglu_sw;
inline int c3i_small_st(const ConvArgs& a, int BM) {
  const long tiles = (long)a.B * a.Ho * a.Wo / BM * ((a.Cout + 63) / 64);
  return tiles <= 256 ? g_c3i_st : 2;
}
inline bool conv3h_pick(const ConvArgs& a) {
  return g_conv3h_on == 2 || (g_conv3h_on == 1 && a.Cin >= 128 && !a.res1 && !a.res2 && !a.bbias);
}

template <typename T, int BM, int BN, int WGM, int WGN, int CK, int ST, int FL = 0, int EPK = EPI_MIN, int WPE = 2>
bool conv3i_try(const ConvArgs& a, hipStream_t st) {
  constexpr int WTM = BM / WGM, BKE = CK / sizeof(T);
  const int RW = conv3_rw(a, BM);
  if (RW <= 0 || RW % WTM || a.Cin % BKE || (a.C1 < a.Cin && a.C1 % BKE)) return false;
  if constexpr ((FL & 1024) != 0) {   // buffer-resource DMA: one row pitch, 31-bit byte offsets
    constexpr size_t LIM = (size_t)1 << 30;
    if (a.x2 && a.C1 < a.Cin && a.ld2 != a.ld1) return false;
    if ((size_t)a.B * a.Hs * a.Ws * a.ld1 * sizeof(T) >= LIM || (size_t)a.Cout * a.K * sizeof(T) >= LIM) return false;
  }
  if constexpr ((FL & 16) != 0)   // fused res_conv: writes y2 from w2, so both must be given
    if (!a.y2 || !a.w2) return false;
  if constexpr ((FL & 8192) != 0) {   // row-phase upsample tiles: one parity per tile
    if (!a.up || !a.uph || a.Ho % (2 * (BM / RW))) return false;
    // column-phase too (FL bit 14): uph == 2, K = 16 Cin, rows of >= 128 output pixels
    if (((FL & 16384) != 0) != (a.uph == 2)) return false;
    if ((FL & 16384) && RW < 128) return false;
  } else if (a.uph) {
    return false;
  }
  if constexpr ((FL & 8) != 0)    // swapped tiles DMA the scale / shift / bias rows in 16-byte pieces
    if ((a.ss && (a.ss_ld % 4 || (a.Cout % 4) || ((uintptr_t)a.ss & 15))) || ((uintptr_t)a.bias & 15)) return false;
  dim3 g(a.B * a.Ho * a.Wo / BM, (a.Cout + BN - 1) / BN, 1);
  conv3i_kernel<T, BM, BN, WGM, WGN, CK, ST, FL, EPK, WPE><<<g, 64 * WGM * WGN, 0, st>>>(a, RW);
  return true;
}
template <typename T>
bool conv3i_launch(int cfg, const ConvArgs& a, hipStream_t st) {
  switch (cfg) {
    case 2: return conv3i_try<T, 256, 64, 4, 1, 64, 2>(a, st);
    case 4: return conv3i_try<T, 128, 128, 2, 2, 64, 2>(a, st);
    case 11: return conv3i_try<T, 256, 64, 4, 1, 64, 2, 1>(a, st);
    case 12: return conv3i_try<T, 256, 64, 4, 1, 64, 2, 2>(a, st);
    case 13: return conv3i_try<T, 256, 64, 4, 1, 64, 2, 3>(a, st);
    case 14: return conv3i_try<T, 256, 128, 4, 2, 64, 2, 1>(a, st);
    case 15: return conv3i_try<T, 256, 128, 4, 2, 64, 2, 3>(a, st);
    case 16: return conv3i_try<T, 256, 64, 4, 1, 64, 3, 1>(a, st);
    case 17: return conv3i_try<T, 256, 64, 4, 1, 64, 2, 5>(a, st);
    case 19: return conv3i_try<T, 64, 128, 2, 2, 64, 2, 4>(a, st);
    case 20: return conv3i_try<T, 128, 64, 4, 1, 64, 2, 4>(a, st);
    case 22: return conv3i_try<T, 64, 64, 2, 1, 64, 2, 4>(a, st);
    case 18: return conv3i_try<T, 256, 64, 4, 1, 64, 2, 4>(a, st);
    case 8: return conv3i_try<T, 128, 128, 4, 2, 64, 3, 3>(a, st);
    case 9: return conv3i_try<T, 128, 128, 4, 2, 64, 2, 3>(a, st);
    case 10: return conv3i_try<T, 128, 64, 4, 1, 64, 2, 3>(a, st);
    case 40:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12>(a, st);
      return false;
    case 41:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 128, 64, 4, 1, 64, 2, 12>(a, st);
      return false;
    case 48:   // 40 / 41 with buffer-resource DMA
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024>(a, st);
      return false;
    case 49:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 128, 64, 4, 1, 64, 2, 12 | 1024>(a, st);
      return false;
    case 52:   // 48 with s_setprio(1) around each stage's MFMAs (FL bit 2)
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 4>(a, st);
      return false;
    case 53:   // 48 with sched_barrier fences around each stage (FL bit 0)
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 1>(a, st);
      return false;
    case 50:   // diagnostic: 48 with every A row read from a 256-pixel (L2-resident) window
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 2048>(a, st);
      return false;
    case 51:   // diagnostic: 50 without the epilogue
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 2048 | 128>(a, st);
      return false;
    case 42:   // diagnostics (convbench only; results are garbage): 40 without DMA / without MFMA
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 32>(a, st);
      return false;
    case 43:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 64>(a, st);
      return false;
    case 44:   // diagnostics: no DMA and no epilogue / no DMA and no barrier / both / no epilogue
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 32 | 128>(a, st);
      return false;
    case 45:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 32 | 256>(a, st);
      return false;
    case 46:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 32 | 128 | 256>(a, st);
      return false;
    case 47:
      if constexpr (sizeof(T) == 2) return a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 128>(a, st);
      return false;
    default: return false;
  }
}

// v5: weight-stationary 3x3 conv for Cin = Cout = 64 (16-bit types), the ResBlock convs of the
// 256x256 / 128x128 levels, whose K = 576 is too short for v4's per-stage weight copies to
// amortise. The block loads all 9 taps x 64 x 64 weights (72 KB) into LDS once and then
// never synchronises again: each of its 8 waves owns a private 2-stage ring holding only its
// own A halo rows (66 pixels x 32 channels per (chunk, kh) stage), so a wave's LDS-DMA wait
// overlaps the other waves' MFMAs instead of stalling the block at a barrier. Waves walk
// 64-pixel row segments persistently (each XCD a contiguous band of rows, for L2 reuse of
// the kh halo rows), and the next segment's first stage is in flight during the epilogue.
// The MFMA operands are swapped (weights as A): with weight row p holding output channel
// 16*((p>>2)&3) + 4*(p>>4) + (p&3), each lane's accumulators are 16 consecutive channels of
// one pixel, so the epilogue runs from registers with 16-byte residual loads and stores.
// Epilogue: (acc + bias) * (1 + scale) + shift -> SiLU -> + res1 + res2 + bbias (EPI_MIN).
// Generalised over (NWV waves, TM = 16-pixel tiles per segment, NST ring stages per wave):
// a deeper private ring keeps NST-1 stages' DMA in flight under the wave's MFMAs (the 2-stage
// ring covered one stage of compute, less than an L2 round trip). LDS: 72 KB of weights +
// NWV * NST * NI KB of rings (NI = DMA instructions of 16 halo rows per stage).
constexpr int C3W_WAVES = 8;
constexpr int C3W_WBYTES = 18 * 64 * 64;            // (chunk, kh, kw) regions of 64 rows x 64 B
template <int NWV, int TM, int NST>
struct C3W {
  static constexpr int SEG = 16 * TM;               // output pixels per segment (tile)
  static constexpr int NI = (SEG + 2 + 15) / 16;    // DMA instructions per stage
  static constexpr int STAGE = NI * 1024;
  static constexpr int SMEM = C3W_WBYTES + NWV * NST * STAGE;
  static_assert(SMEM <= 160 * 1024, "LDS");
};
// BUF: the halo DMA through a raw buffer descriptor whose base sits one pixel before the input,
// with every per-lane offset a kernel-lifetime constant (halo column x row pitch + slot) and the
// segment's row / column start in the scalar soffset; padding lanes (image edges, rows past the
// halo, rows outside the image, tiles past the wave's range) carry an out-of-range offset the
// range check lands as zeros. No per-stage address arithmetic and no branches around the DMA
// (the flat form spent ~55 VALU per stage there). Needs one row pitch (ld2 == ld1 when split).
template <typename T, int NWV, int TM = 4, int NST = 2, bool BUF = false, bool Q8 = false>
__global__ void __launch_bounds__(64 * NWV) conv3w_kernel(ConvArgs a, int ntiles, int delay) {
  kernarg_touch<sizeof(ConvArgs) + 8>();                     // every kernarg line once, one wait (common.h)
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  using CF = C3W<NWV, TM, NST>;
  constexpr int NF = TM + 2, VE = 8, SEG = CF::SEG, NI = CF::NI, STAGE = CF::STAGE;
  using SA = RowSwz<4, TM>;
  using SB = RowSwz<4, 1>;
  __shared__ __attribute__((aligned(1024))) char smem[CF::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const char* zero = reinterpret_cast<const char*>(a.zero);

  // Weights -> LDS, once. DMA instruction q fills region q/4 (= (c*3 + kh)*3 + kw), rows
  // (q%4)*16 + lane/4, 16-byte physical slot lane%4.
  for (int q = wave; q < 72; q += NWV) {
    const int g = q >> 2, rho = (q & 3) * 16 + (lane >> 2);
    const int c = g / 9, tap = g % 9;
    const int n = wperm64(rho);
    const int L = SB::slot(rho, lane & 3);
    const T* src = reinterpret_cast<const T*>(a.w) + (size_t)n * a.K + tap * 64 + c * 32 + L * VE;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(smem + q * 1024), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Tiles of this wave: XCD band [x*ntiles/8, (x+1)*ntiles/8), strided over the band's waves.
  const int xcd = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int t_end = (int)((long)(xcd + 1) * ntiles / 8);
  const int stride = nbx * NWV;
  int t = (int)((long)xcd * ntiles / 8) + (blockIdx.x >> 3) * NWV + wave;
  if (t >= t_end) return;

  char* ring = smem + C3W_WBYTES + wave * NST * STAGE;
  const char* wl = smem;
  const int segs = a.Wo / SEG;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  // Per-lane DMA geometry: instruction j fills physical halo row j*16 + lane/4.
  int dr[NI], dls[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int R = SA::logical(j * 16 + (lane >> 2));
    dr[j] = R;
    dls[j] = SA::slot(R, lane & 3) * VE * 2;
  }
  int aoff[NF], boff[4];
#pragma unroll
  for (int s = 0; s < NF; ++s) aoff[s] = SA::phys(TM * lr + s) * 64 + (SA::slot(TM * lr + s, lg) << 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) boff[j] = (16 * j + lr) * 64 + (SB::slot(16 * j + lr, lg) << 4);

  // BUF per-lane constants: byte offset of halo row R = dr (output column ow0 + R - 1, source
  // column (ow0 >> up) + ((R - 1) >> up)) from the pixel before the segment's first source pixel.
  constexpr unsigned OOB = 0x80000000u;
  int boffs[BUF ? NI : 1];
  const int up = a.up ? 1 : 0;
  const int x_bytes = BUF ? a.B * a.Hs * a.Ws * a.ld1 * 2 + a.ld1 * 2 : 0;
  if constexpr (BUF) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      boffs[j] = dr[j] < SEG + 2 ? (int)((((dr[j] - 1) >> up) + 1) * a.ld1 * 2 + dls[j]) : (int)OOB;
  }
  // Stage (c, kh) of tile tt into ring slot `slot`; tiles past this wave's range load the zero
  // page so every stage issues exactly NI instructions (the counted waits rely on it).
  auto issue = [&](int tt, int c, int kh, int slot) {
    if constexpr (BUF) {
      const bool live = tt < t_end;
      const int rr = live ? tt / segs : 0, ow0 = live ? (tt - rr * segs) * SEG : 0;
      const int b = rr / a.Ho, oh = rr - b * a.Ho;
      const int ih = oh + kh - 1;
      const int ci0 = c * 32;
      const bool from1 = ci0 < a.C1;
      const bool row_ok = live && (unsigned)ih < (unsigned)Hin;
      const int prow = b * a.Hs + (a.up ? (ih >> 1) : ih);
      const int soff = row_ok ? ((prow * a.Ws + (ow0 >> up)) * a.ld1 + (from1 ? ci0 : ci0 - a.C1)) * 2 : 0;
      const char* base = reinterpret_cast<const char*>(from1 ? a.x1 : a.x2) - a.ld1 * 2;
      const bool lpad = ow0 == 0, rpad = ow0 + SEG == a.Wo;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int vo = row_ok ? boffs[j] : (int)OOB;
        if (j == 0) vo = (lpad && dr[j] == 0) ? (int)OOB : vo;
        if ((SEG + 1) / 16 == j) vo = (rpad && dr[j] == SEG + 1) ? (int)OOB : vo;
        buf_lds16(base, x_bytes, ring + slot * STAGE + j * 1024, vo, soff);
      }
      return;
    }
    const bool live = tt < t_end;
    const int rr = live ? tt / segs : 0, ow0 = live ? (tt - rr * segs) * SEG : 0;
    const int b = rr / a.Ho, oh = rr - b * a.Ho;
    const int ih = oh + kh - 1;
    const int ci0 = c * 32;
    const bool from1 = ci0 < a.C1;
    const char* xs = reinterpret_cast<const char*>(from1 ? a.x1 : a.x2) + (size_t)(from1 ? ci0 : ci0 - a.C1) * 2;
    const size_t ldb = (size_t)(from1 ? a.ld1 : a.ld2) * 2;
    const bool row_ok = live && (unsigned)ih < (unsigned)Hin;
    const int prow = b * a.Hs + (a.up ? (ih >> 1) : ih);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int iw = ow0 + dr[j] - 1;
      const char* src = zero;
      if (row_ok && dr[j] < SEG + 2 && (unsigned)iw < (unsigned)Win)
        src = xs + ((size_t)prow * a.Ws + (a.up ? (iw >> 1) : iw)) * ldb + dls[j];
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(ring + slot * STAGE + j * 1024), 16, 0, 0);
    }
  };

  const int nb = 16 * lg;
  float bi[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) bi[e] = a.bias ? a.bias[nb + e] : 0.f;

  // Waves 4-7 share SIMDs with waves 0-3: start them about half a segment later, so one
  // wave's epilogue (VALU, SiLU transcendentals) overlaps its SIMD partner's MFMA phase.
  if (NWV > 4 && (wave & 4))
    for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(8);
  // Global stage g = 6 * (tile index along this wave's walk) + (c * 3 + kh) lands in slot
  // g % NST; stages g+1 .. g+NST-1 are in flight while g computes.
#pragma unroll
  for (int q = 0; q < NST - 1; ++q) issue(t + (q / 6) * stride, (q % 6) / 3, q % 3, q);
  int slot = 0;
  int g = 0;
  while (true) {
    const int tn = t + stride;
    const int rr = t / segs;
    const int b = rr / a.Ho;
    const int m0 = rr * a.Wo + (t - rr * segs) * SEG;
    f32x4 acc[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    EpiPref<TM> pref;
#pragma unroll
    for (int s = 0; s < 6; ++s, ++g) {
      const int c = s / 3, kh = s % 3;
      // Own DMA of stage g landed: NST-2 younger stages (NI instructions each) may stay in
      // flight. At a tile's first stage the previous tile's epilogue issued its 2*TM 16-byte
      // stores after this stage's DMA (vmcnt retires in issue order), so those may stay in
      // flight too instead of stalling the wave for a store round trip.
      if constexpr (NST == 2) {
        if (s == 0 && g > 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(2 * TM) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"((NST - 2) * NI) : "memory");
      }
      if (s == 5) epi_prefetch<T, TM>(a, nb, b, [&](int i) { return (size_t)m0 + TM * lr + i; }, pref);
      {
        const int sn = s + NST - 1;                   // stage to issue: (tile + sn/6, sn%6)
        issue(t + (sn / 6) * stride, (sn % 6) / 3, sn % 3, (slot + NST - 1) % NST);
      }

      const char* st = ring + slot * STAGE;
      u32x4 fa[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) fa[f] = *reinterpret_cast<const u32x4*>(st + aoff[f]);
      // Weight fragments double-buffered across the kw taps: tap kw+1's reads are in flight
      // under tap kw's MFMAs.
      const char* wr0 = wl + (c * 3 + kh) * 3 * 4096;
      u32x4 fw[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fw[0][j] = *reinterpret_cast<const u32x4*>(wr0 + boff[j]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        if (kw < 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) fw[(kw + 1) & 1][j] = *reinterpret_cast<const u32x4*>(wr0 + (kw + 1) * 4096 + boff[j]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], fw[kw & 1][j], fa[i + kw]);
      }
      slot = slot + 1 == NST ? 0 : slot + 1;
    }
    // Epilogue: tile i of lane (lr, lg) is pixel m0 + TM*lr + i, channels nb .. nb+15. The
    // prefetched operands landed once at most the next tile's first stage (NI DMA) is pending.
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI) : "memory");
    epi_regs16<T, TM, false, true, Q8>(a, acc, bi, nb, b, [&](int i) { return (size_t)m0 + TM * lr + i; }, &pref);
    if (tn >= t_end) break;
    t = tn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------
// v6 (3x3, stride 1, pad 1, 16-bit): 2-D halo tiles, one stage per 32-channel chunk.
// A tile is 8 output rows x 64 columns of one image x 64 output channels; wave w (of 8) owns
// output row w (64 pixels, TM = 4 interleaved 16-pixel MFMA tiles as in v4) x all 64 channels
// (swapped operands: weights as the MFMA A operand, so each lane ends with 16 consecutive
// channels of one pixel and the register epilogue epi_regs16 writes them).
// One stage holds, for one 32-channel chunk, the whole 10 x 66 input halo of the tile (each
// input pixel landed in LDS once per chunk, not once per kh as in v4's (chunk, kh) stages)
// and all 9 weight taps (576 rows): 78 KB, two stages + two epilogue-term slots = 158 KB, one
// block of 8 waves per CU. Per stage a wave reads 3 x (6 A + 3 x 4 B) fragments and issues 144
// MFMAs; one barrier per stage (v4: one per 48 MFMAs). LDS-DMA bytes per output are 0.46x v4's
// (v4's 256 x 64 tiles re-fetch the halo for every kh and the taps for every 256 pixels), which
// takes the CU's LDS-DMA landing rate off the critical path.
// Persistent: each block walks tiles of its XCD's contiguous tile range (n-tile fastest, so
// the blocks of an XCD share halo rows in L2); the next tile's first stage (and its epilogue
// terms) is DMA'd at the last stage's barrier, under that stage's MFMAs and the epilogue.
// Buffer-descriptor DMA with out-of-range zero fill for the padding (as v4 FL bit 10).
constexpr int C3H_RH = 8, C3H_RW = 64, C3H_HWID = C3H_RW + 2;
constexpr int C3H_NPIX = (C3H_RH + 2) * C3H_HWID;              // 660 halo pixels
constexpr int C3H_NA = (C3H_NPIX + 15) / 16;                    // 42 A DMA instructions
constexpr int C3H_NB = 9 * 64 / 16;                             // 36 B DMA instructions
constexpr int C3H_STAGE = (C3H_NA + C3H_NB) * 1024;             // 79872 B
constexpr int C3H_SMEM = 2 * C3H_STAGE + 2 * 1024;              // + 2 epilogue-term slots
static_assert(C3H_SMEM <= 160 * 1024, "v6 LDS");
inline int conv3h_ntiles(const ConvArgs& a) { return a.B * (a.Ho / C3H_RH) * (a.Wo / C3H_RW) * (a.Cout / 64); }

// FL bit 0 (the default): the stage's LDS-DMA is issued in three parts, one after each kh's
// MFMAs, instead of all at the stage start, where every wave of the block issues at once right
// after the barrier (3-8 % faster; starting the blocks out of phase was 5-20 % slower).
template <typename T, int FL = 1>
__global__ void __launch_bounds__(512) conv3h_kernel(ConvArgs a, int ntiles) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int TM = 4, NF = TM + 2, VE = 8, ES = 2;
  constexpr unsigned OOB = 0x80000000u;
  using SA = RowSwz<4, TM>;
  using SB = RowSwz<4, 1>;
  static_assert(C3H_NPIX % 4 == 0, "A rows: whole permutation groups");
  __shared__ __attribute__((aligned(1024))) char smem[C3H_SMEM];
  char* terms = smem + 2 * C3H_STAGE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int HWo = a.Ho * a.Wo;
  const int NT = a.Cout / 64, cols = a.Wo / C3H_RW, tiles_img = (a.Ho / C3H_RH) * cols;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  const int x_bytes = a.B * a.Hs * a.Ws * a.ld1 * ES, w_bytes = a.Cout * a.K * ES;
  const int nchunk = a.Cin / 32;

  // This block's tiles: XCD x's contiguous range [x*ntiles/8, (x+1)*ntiles/8), dealt round-robin
  // to the blocks of that XCD (blocks b and b+8 share one; speed only).
  const int nb = gridDim.x, xcd = blockIdx.x & 7, jx = blockIdx.x >> 3, cx = (nb - xcd + 7) >> 3;
  const int t_beg = (int)((long)xcd * ntiles / 8), t_end = (int)((long)(xcd + 1) * ntiles / 8);
  int t = t_beg + jx;
  if (t >= t_end) return;

  struct Tile { int b, oh0, ow0, n0; };
  auto tile_of = [&](int tt) {
    Tile o;
    const int sp = tt / NT;
    o.n0 = (tt - sp * NT) * 64;
    o.b = sp / tiles_img;
    const int r = sp - o.b * tiles_img;
    o.oh0 = (r / cols) * C3H_RH;
    o.ow0 = (r - (r / cols) * cols) * C3H_RW;
    return o;
  };
  // Per-tile DMA tables of this wave: A instruction q = wave + 8j (< 42) fills physical halo rows
  // 16q .. 16q+15 (lane / 4), B instruction q = wave + 8j (< 36) weight rows 16q .. (tap = row / 64).
  int a_off[6], b_off[5];
  auto tables = [&](const Tile& tl) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int q = wave + 8 * j;
      const int P = q * 16 + (lane >> 2);
      const int R = SA::logical(P);
      const int hy = R / C3H_HWID, hx = R - hy * C3H_HWID;
      const int ih = tl.oh0 + hy - 1, iw = tl.ow0 + hx - 1;
      const bool ok = q < C3H_NA && R < C3H_NPIX && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win;
      const int pix = tl.b * a.Hs * a.Ws + (a.up ? (ih >> 1) : ih) * a.Ws + (a.up ? (iw >> 1) : iw);
      a_off[j] = ok ? (pix * a.ld1 + SA::slot(R, lane & 3) * VE) * ES : (int)OOB;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int q = wave + 8 * j;
      const int row = q * 16 + (lane >> 2);
      const int tap = row >> 6, n = tl.n0 + wperm64(row & 63);
      b_off[j] = q < C3H_NB ? (int)(((size_t)n * a.K + tap * a.Cin + SB::slot(row, lane & 3) * VE) * ES) : (int)OOB;
    }
  };
  // Pieces [p0, p1) of this wave's 11 DMA instructions (6 A, then 5 B) of stage (tl, c).
  auto issue_part = [&](const Tile& tl, int c, int slot, int p0, int p1) {
    char* st = smem + slot * C3H_STAGE;
    const int ci0 = c * 32;
    const bool from1 = ci0 < a.C1;
    const void* xb = from1 ? a.x1 : a.x2;
    const int soa = (from1 ? ci0 : ci0 - a.C1) * ES;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j >= p0 && j < p1 && wave + 8 * j < C3H_NA) buf_lds16(xb, x_bytes, st + (wave + 8 * j) * 1024, a_off[j], soa);
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (6 + j >= p0 && 6 + j < p1 && wave + 8 * j < C3H_NB)
        buf_lds16(a.w, w_bytes, st + (C3H_NA + wave + 8 * j) * 1024, b_off[j], ci0 * ES);
  };
  auto issue = [&](const Tile& tl, int c, int slot, bool with_terms, int tslot) {
    issue_part(tl, c, slot, 0, 11);
    if (with_terms && wave == 0) {                 // lanes 0-15 scale, 16-31 shift, 32-47 bias
      const int part = lane >> 4, l16 = lane & 15;
      const float* src = reinterpret_cast<const float*>(a.zero);
      if (part == 0 && a.ss) src = a.ss + (size_t)tl.b * a.ss_ld + tl.n0 + 4 * l16;
      else if (part == 1 && a.ss) src = a.ss + (size_t)tl.b * a.ss_ld + a.Cout + tl.n0 + 4 * l16;
      else if (part == 2 && a.bias) src = a.bias + tl.n0 + 4 * l16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(terms + tslot * 1024), 16, 0, 0);
    }
  };

  // Fragment offsets (stage-relative): A for (kh, s): halo row (wave + kh) * 66 + TM*lr + s.
  int aoff[3][NF];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int s2 = 0; s2 < NF; ++s2) {
      const int R = (wave + kh) * C3H_HWID + TM * lr + s2;
      aoff[kh][s2] = SA::phys(R) * 64 + (SA::slot(R, lg) << 4);
    }
  int boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 16 * j + lr;
    boff[j] = C3H_NA * 1024 + row * 64 + (SB::slot(row, lg) << 4);   // + tap * 4096
  }

  // (Residual-row prefetch into registers, as v4 / v5 do, does not fit the register budget.)
  constexpr bool pre_ok = false;
  Tile cur = tile_of(t);
  tables(cur);
  issue(cur, 0, 0, true, 0);
  int g = 0, k = 0;
  while (true) {
    const int tn = t + cx;
    const bool has_next = tn < t_end;
    const Tile nxt = has_next ? tile_of(tn) : cur;
    f32x4 acc[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    EpiPref<TM> pref;
    const size_t rowbase = (size_t)cur.b * HWo + (size_t)(cur.oh0 + wave) * a.Wo + cur.ow0;
    auto pixf = [&](int i) { return rowbase + TM * lr + i; };
    for (int c = 0; c < nchunk; ++c, ++g) {
      // Own DMA of stage g landed. At a tile's first stage (after the first tile) the previous
      // epilogue's 2*TM stores are younger than it and may stay in flight.
      if (c == 0 && k > 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(2 * TM) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // Next stage: (cur, c + 1), or the next tile's first chunk (with its terms) at the last.
      const bool nx = c + 1 < nchunk || has_next;
      const Tile& tn2 = c + 1 < nchunk ? cur : nxt;
      const int cn = c + 1 < nchunk ? c + 1 : 0;
      if (c + 1 == nchunk && has_next) tables(nxt);
      if constexpr ((FL & 1) == 0) {
        if (nx) issue(tn2, cn, (g + 1) & 1, c + 1 == nchunk, (k + 1) & 1);
      } else if (nx && c + 1 == nchunk && wave == 0) {   // terms now; the DMA pieces follow the MFMAs
        const int part = lane >> 4, l16 = lane & 15;
        const float* src = reinterpret_cast<const float*>(a.zero);
        if (part == 0 && a.ss) src = a.ss + (size_t)tn2.b * a.ss_ld + tn2.n0 + 4 * l16;
        else if (part == 1 && a.ss) src = a.ss + (size_t)tn2.b * a.ss_ld + a.Cout + tn2.n0 + 4 * l16;
        else if (part == 2 && a.bias) src = a.bias + tn2.n0 + 4 * l16;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(terms + ((k + 1) & 1) * 1024), 16, 0, 0);
      }
      if (c + 1 == nchunk && pre_ok) epi_prefetch<T, TM>(a, cur.n0 + 16 * lg, cur.b, pixf, pref);
      const char* st = smem + (g & 1) * C3H_STAGE;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        u32x4 fa[NF];
#pragma unroll
        for (int s2 = 0; s2 < NF; ++s2) fa[s2] = *reinterpret_cast<const u32x4*>(st + aoff[kh][s2]);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const char* sb = st + (kh * 3 + kw) * 4096;
          u32x4 fb[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const u32x4*>(sb + boff[j]);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], fb[j], fa[i + kw]);
        }
        if constexpr ((FL & 1) != 0)
          if (nx) issue_part(tn2, cn, (g + 1) & 1, 4 * kh, kh == 2 ? 11 : 4 * kh + 4);
      }
    }
    // Epilogue of this tile (terms slot k & 1 landed with its first stage).
    if (pre_ok) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int nbch = cur.n0 + 16 * lg;
    const float* el = reinterpret_cast<const float*>(terms + (k & 1) * 1024) + 16 * lg;
    float bi[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bi[e] = el[128 + e];
    if (pre_ok) epi_regs16<T, TM, false, true>(a, acc, bi, nbch, cur.b, pixf, &pref, el);
    else epi_regs16<T, TM>(a, acc, bi, nbch, cur.b, pixf, nullptr, el);
    if (!has_next) break;
    t = tn;
    cur = nxt;
    ++k;
  }
}

template <typename T>
void conv3h_launch(const ConvArgs& a, hipStream_t st, int fl = 0) {
  const int nt = conv3h_ntiles(a);
  const int grid = nt < 256 ? nt : 256;
  if (fl == 0) conv3h_kernel<T, 0><<<grid, 512, 0, st>>>(a, nt);
  else conv3h_kernel<T, 1><<<grid, 512, 0, st>>>(a, nt);
}

// Kernel shape of the 64 -> 64 3x3 convs: DAC_C3W=<waves>,<TM>,<stages> (tuning), default
// 8 waves x 64-pixel segments x 2 stages.
struct C3WCfg { int nwv = 8, tm = 4, nst = 2; };
// Small grids (fewer 64-pixel segments than two per wave of a full-chip launch: the 128x128
// level) may take another shape (DAC_C3W_SMALL); DAC_C3W forces one shape everywhere.
constexpr C3WCfg kC3WSmall{8, 4, 2};
inline C3WCfg c3w_cfg(bool small = false) {
  static C3WCfg c = [] {
    C3WCfg r;
    if (const char* e = getenv("DAC_C3W")) sscanf(e, "%d,%d,%d", &r.nwv, &r.tm, &r.nst);
    return r;
  }();
  static C3WCfg cs = [] {
    C3WCfg r = kC3WSmall;
    if (const char* e = getenv("DAC_C3W")) sscanf(e, "%d,%d,%d", &r.nwv, &r.tm, &r.nst);
    else if (const char* e2 = getenv("DAC_C3W_SMALL")) sscanf(e2, "%d,%d,%d", &r.nwv, &r.tm, &r.nst);
    return r;
  }();
  return small ? cs : c;
}
inline int conv3w_blocks(int ntiles, int nwv) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      ncu = 256;
  }
  int nb = (ntiles + nwv - 1) / nwv;
  if (nb > ncu) nb = ncu;
  return (nb + 7) / 8 * 8;                          // whole XCD bands
}
template <typename T>
void conv3w_launch(const ConvArgs& a, int delay, hipStream_t st) {
  const C3WCfg c = c3w_cfg(a.Wo % 64 == 0 && (long)a.B * a.Ho * (a.Wo / 64) < 2L * 256 * C3W_WAVES);
#define DAC_C3W(NW_, TM_, NS_)                                                                 \
  if (!a.ys8 && c.nwv == NW_ && c.tm == TM_ && c.nst == NS_ && a.Wo % (16 * TM_) == 0) {       \
    const int ntiles = a.B * a.Ho * (a.Wo / (16 * TM_));                                        \
    conv3w_kernel<T, NW_, TM_, NS_><<<conv3w_blocks(ntiles, NW_), 64 * NW_, 0, st>>>(a, ntiles, delay); \
    return;                                                                                     \
  }
  DAC_C3W(8, 2, 3)
  DAC_C3W(8, 2, 2)
  DAC_C3W(4, 4, 4)
  DAC_C3W(4, 4, 3)
  DAC_C3W(6, 4, 2)
#undef DAC_C3W
  const int ntiles = a.B * a.Ho * (a.Wo >> 6);
  // Buffer-descriptor DMA when the input has one row pitch and 31-bit byte offsets.
  static const int buf_env = getenv("DAC_C3W_BUF") ? atoi(getenv("DAC_C3W_BUF")) : 1;
  const bool buf = buf_env && (a.C1 >= a.Cin || !a.x2 || a.ld2 == a.ld1) &&
                   (size_t)a.B * a.Hs * a.Ws * a.ld1 * 2 + a.ld1 * 2 < ((size_t)1 << 31);
  if (a.ys8) {                                      // fp8 output (conv_q8out_ok): buffer DMA form only
    if (!buf) throw std::logic_error("conv3w: fp8 output needs the buffer-descriptor DMA form");
    conv3w_kernel<T, C3W_WAVES, 4, 2, true, true><<<conv3w_blocks(ntiles, C3W_WAVES), 64 * C3W_WAVES, 0, st>>>(a, ntiles, delay);
  } else if (buf)
    conv3w_kernel<T, C3W_WAVES, 4, 2, true><<<conv3w_blocks(ntiles, C3W_WAVES), 64 * C3W_WAVES, 0, st>>>(a, ntiles, delay);
  else
    conv3w_kernel<T, C3W_WAVES, 4, 2><<<conv3w_blocks(ntiles, C3W_WAVES), 64 * C3W_WAVES, 0, st>>>(a, ntiles, delay);
}

// v3 launch, buffer-descriptor DMA when the input has one row pitch and 30-bit byte offsets.
template <typename T, int BM, int BN, int WGM, int WGN, int CK>
void conv3_launch(const ConvArgs& a, dim3 g, int RW, hipStream_t st) {
  constexpr size_t LIM = (size_t)1 << 30;
  const bool buf = g_conv3_buf && (a.C1 >= a.Cin || !a.x2 || a.ld2 == a.ld1) &&
                   (size_t)a.B * a.Hs * a.Ws * a.ld1 * sizeof(T) < LIM && (size_t)a.Cout * a.K * sizeof(T) < LIM;
  if (buf) conv3_kernel<T, BM, BN, WGM, WGN, CK, true><<<g, 64 * WGM * WGN, 0, st>>>(a, RW);
  else conv3_kernel<T, BM, BN, WGM, WGN, CK><<<g, 64 * WGM * WGN, 0, st>>>(a, RW);
}

template <typename T, int KH, int KW, int S, int P>
void conv_dispatch(const ConvArgs& a0, hipStream_t st) {
  // 1x1 GEMMs: buffer-descriptor DMA when the input has one row pitch and every byte offset
  // fits 31 bits (ConvArgs::dbuf; DAC_CONV3_BUF=0 disables it with the 3x3 forms).
  ConvArgs a = a0;
  a.dbuf = 0;
  if constexpr (KH == 1 && KW == 1 && S == 1 && P == 0) {
    constexpr size_t LIM = (size_t)1 << 31;
    const size_t es = sizeof(T);
    a.dbuf = g_conv3_buf && (!a.x2 || a.C1 >= a.Cin || a.ld2 == a.ld1) && !a.up &&
             (size_t)a.B * a.Hs * a.Ws * a.ld1 * es < LIM && (!a.x2 || (size_t)a.B * a.Hs * a.Ws * a.ld2 * es < LIM) &&
             (size_t)a.Cout * a.K * es < LIM;
  }
  // A fused second output is only requested after conv_res_fusable(a) said the v4 path takes it;
  // no path below may return without writing it.
  if (a.y2 && !(KH == 3 && KW == 3 && S == 1 && P == 1 && sizeof(T) == 2 && conv_res_fusable(a)))
    throw std::logic_error("conv: fused second output requested on a shape without a fusing kernel");
  const int M = a.B * a.Ho * a.Wo;
  const bool batched = a.w_bstride > 0;
  const int Mg = batched ? a.Ho * a.Wo : M;
  const int gz = batched ? a.B : 1;
  constexpr int BKE = 128 / sizeof(T);
  // Tap shapes whose Cin is always a multiple of the K tile use v2; v1 serves the rest
  // (init conv Cin=8, patch embed, final conv Cout=3, LinearAttention to_out amode=1).
  constexpr bool V2 = (KH == 1 || KH == 3 || KH == 4);
  const bool v2ok = V2 && a.zero != nullptr && a.Cin % BKE == 0 && a.amode == 0 && a.Cout > 16;
  if constexpr (KH == 3 && KW == 3 && S == 1 && P == 1) {
    if (a.ksplit > 1 && a.part) {
      // Split-K (engine conv_call; conv3_split_ok): v3's 8-wave 128 x 128 form over ksplit Cin
      // ranges (grid z), then the in-order reduce + epilogue pass.
      if (!conv3_split_ok(a, (int)sizeof(T))) throw std::invalid_argument("conv: 3x3 split-K on a shape without it");
      dim3 g(a.B * a.Ho * a.Wo / 128, (a.Cout + 127) / 128, a.ksplit);
      conv3_launch<T, 128, 128, 4, 2, 128>(a, g, conv3_rw(a, 128), st);
      conv_part_reduce<T>(a, st);
      return;
    }
  }
  if constexpr (KH == 3 && KW == 3 && S == 1 && P == 1 && sizeof(T) == 2) {
    if (g_conv3_force < 0 && conv3n_ok(a)) {   // final_conv: conv_edge.hip
      conv3n<T>(a, st);
      return;
    }
  }
  if constexpr (KH == 3 && KW == 3 && S == 1 && P == 1) {
    // Narrow output (the final conv, Cout = 3): v4 row-halo tiles with 16 output channels and
    // the general (scalar-capable) epilogue; the A operand dominates, and v4 reads each input
    // pixel once per kernel row instead of 9 times.
    if (a.Cout <= 16 && a.zero && a.amode == 0 && a.w_bstride == 0 && g_conv3_force < 0 &&
        (a.act == ACT_NONE || a.act == ACT_SILU) && a.Cin % (64 / (int)sizeof(T)) == 0)
      if (conv3i_try<T, 256, 16, 4, 1, 64, 2, 3, EPI_ALL>(a, st)) return;
  }
  if constexpr (KH == 3 && KW == 3 && S == 1 && P == 1 && sizeof(T) == 2) {
    // v6 (2-D halo tiles): force 60, or DAC_CONV3H=1 for every shape it takes.
    // v6 (2-D halo tiles): forces 60 / 61 (without / with the interleaved DMA issue); by default
    // (DAC_CONV3H=1) the plain convs with Cin >= 128 it measured faster on,
    // DAC_CONV3H=2 every shape it takes, 0 none.
    if (((g_conv3_force == 60 || g_conv3_force == 61) ||
         (g_conv3_force < 0 && conv3h_pick(a))) && conv3h_ok(a, (int)sizeof(T))) {
      conv3h_launch<T>(a, st, g_conv3_force == 60 ? 0 : 1);
      return;
    }
    if ((g_conv3_force < 0 || g_conv3_force == 70) && conv3r_ok(a)) {
      conv3r<T>(a, st);
      return;
    }
    if ((g_conv3_force < 0 || (g_conv3_force >= 30 && g_conv3_force < 40)) && conv3w_ok(a)) {
      const int delay = g_conv3_force >= 30 ? (g_conv3_force - 30) * 2 : 6;   // swept: 4-10 best
      conv3w_launch<T>(a, delay, st);
      return;
    }
  }
  if constexpr (KH == 4 && KW == 4 && S == 2 && P == 1 && sizeof(T) == 2) {
    if (g_conv3_force < 0 && conv_down_ok(a)) {
      conv_down<T>(a, st);
      return;
    }
  }
  if constexpr (KH == 7 && KW == 7 && S == 1 && P == 3 && sizeof(T) == 2) {
    if (conv7_ok(a)) {
      conv7<T>(a, st);
      return;
    }
    if (a.Cin == 8 && a.K == (a.cwrap ? 2 : 1) * 7 * 8 * 8 && a.zero && a.amode == 0 && a.w_bstride == 0 && !a.x2) {
      const int Mg = a.B * a.Ho * a.Wo;
      dim3 g((Mg + 255) / 256, (a.Cout + 63) / 64, 1);
      conv2_kernel<T, 256, 64, 4, 2, 3, KH, KW, S, P, EPI_ALL><<<g, 512, 0, st>>>(a);
      return;
    }
    // cwrap = 1 here means the row-tap dual layout (kernel rows wrap); the generic loaders read
    // a nonzero cwrap as a channel wrap instead, so no other kernel may take it.
    if (a.cwrap) throw std::logic_error("conv: 7x7 row-tap dual layout without its kernel");
  }
  if constexpr (KH == 3 && KW == 3 && S == 1 && P == 1) {
    const int RW = conv3_rw(a);
    // v3's epilogue is compiled for the fast case only: SiLU / none, 16-byte rows.
    const bool epi_min = (a.act == ACT_NONE || a.act == ACT_SILU) && a.Cout % (16 / (int)sizeof(T)) == 0 &&
                         a.ldy % (16 / (int)sizeof(T)) == 0 && (!a.res1 || a.ldr1 % (16 / (int)sizeof(T)) == 0) &&
                         (!a.res2 || a.ldr2 % (16 / (int)sizeof(T)) == 0);
    if (v2ok && RW > 0 && a.w_bstride == 0 && epi_min && a.cwrap == 0) {
      if (g_conv3_force > 0) {
        if (conv3i_launch<T>(g_conv3_force, a, st)) return;
      } else if (g_conv3_force < 0) {
        // v4: 256 x 64 tiles, 4 waves of 64x64, interleaved rows (measured 3-15 % faster than
        // v3 at every 3x3 shape of the UNet whose row width is a multiple of 64).
        // bf16 with whole 64-channel tiles: swapped operands + register epilogue (FL bit 3),
        // 4-9 % faster than the LDS-staged epilogue at every v4 shape of the UNet.
        if constexpr (sizeof(T) == 2) {
          // Buffer-resource DMA (FL bit 10) first; the flat-address form takes what it rejects.
          const int nb = g_conv3_buf ? 1024 : 0;
          if (a.uph) {                                // row- (and column-) phase upsample conv (conv_uph_ok)
            if (a.uph == 2 && nb && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 8192 | 16384>(a, st)) return;
            if (a.uph == 2 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 8192 | 16384>(a, st)) return;
            if (a.uph == 1 && nb && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024 | 8192>(a, st)) return;
            if (a.uph == 1 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 8192>(a, st)) return;
            throw std::logic_error("conv: row-phase upsample conv without a matching v4 tile");
          }
          if (a.ys8) {                                // fp8 output (conv_q8out_ok): fused-res tiles only
            if (a.y2 && a.Cout == 64 && nb && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 16 | 1024 | 4096>(a, st)) return;
            if (a.y2 && a.Cout == 64 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 16 | 4096>(a, st)) return;
            throw std::logic_error("conv: fp8 output without a matching fused v4 tile");
          }
          if (a.y2) {
            if (a.Cout % 64 == 0 && nb && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 16 | 1024>(a, st)) return;
            if (a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 16>(a, st)) return;
            if (a.Cout % 64 == 0 && nb && conv3i_try<T, 128, 64, 4, 1, 64, 2, 12 | 16 | 1024>(a, st)) return;
            if (a.Cout % 64 == 0 && conv3i_try<T, 128, 64, 4, 1, 64, 2, 12 | 16>(a, st)) return;
            throw std::logic_error("conv: conv_res_fusable promised a fused kernel");
          } else if (a.Cout % 64 == 0 && nb && c3i_small_st(a, 256) == 3 && conv3i_try<T, 256, 64, 4, 1, 64, 3, 12 | 1024>(a, st)) {
            return;
          } else if (a.Cout % 64 == 0 && nb && c3i_small_st(a, 256) == 4 && conv3i_try<T, 256, 64, 4, 1, 64, 4, 12 | 1024>(a, st)) {
            return;
          } else if (a.Cout % 64 == 0 && nb && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12 | 1024>(a, st)) {
            return;
          } else if (a.Cout % 64 == 0 && conv3i_try<T, 256, 64, 4, 1, 64, 2, 12>(a, st)) {
            return;
          }
        }
        if (conv3i_try<T, 256, 64, 4, 1, 64, 2, 4>(a, st)) return;
        // Rows of 32 (the 32x32 level), Cout <= 256: 128x64 tiles of 32-pixel wave tiles
        // (TM = 2), 8 % faster than v3 in the UNet; the 512-wide convs stay on v3 (v4 with
        // 128x128 tiles measured 3-4 % slower there).
        // (The 512-wide convs stay on v3: v4 128x64 swapped tiles measured 11 % faster in
        // convbench but 3 % slower in the network.)
        if constexpr (sizeof(T) == 2)
          if (a.Cout <= 256 && a.Cout % 64 == 0) {
            if (g_conv3_buf && c3i_small_st(a, 128) == 3 && conv3i_try<T, 128, 64, 4, 1, 64, 3, 12 | 1024>(a, st)) return;
            if (g_conv3_buf && c3i_small_st(a, 128) == 4 && conv3i_try<T, 128, 64, 4, 1, 64, 4, 12 | 1024>(a, st)) return;
            if (g_conv3_buf && conv3i_try<T, 128, 64, 4, 1, 64, 2, 12 | 1024>(a, st)) return;
            if (conv3i_try<T, 128, 64, 4, 1, 64, 2, 12>(a, st)) return;
          }
        if (a.Cout <= 256 && conv3i_try<T, 128, 64, 4, 1, 64, 2, 4>(a, st)) return;
      }
      // 64-byte K rows, 4 waves of 64x64 (or 64x32) wave tiles: two 24-36 KB stages, so 2-3
      // blocks share a CU and one block's LDS-DMA latency hides behind another's MFMAs
      // (measured 10-24 % faster than one 8-wave block with 128-byte rows). Small grids
      // (< 2 blocks per CU, the 32x32 level) keep the 8-wave block.
      if (a.Cout <= 64 && conv3_rw(a, 128) > 0) {
        dim3 g(a.B * a.Ho * a.Wo / 128, (a.Cout + 63) / 64, 1);
        conv3_launch<T, 128, 64, 2, 2, 64>(a, g, conv3_rw(a, 128), st);
        return;
      }
      if (a.Cout <= 64) {
        dim3 g(a.B * a.Ho * a.Wo / 256, (a.Cout + 63) / 64, 1);
        conv3_launch<T, 256, 64, 4, 2, 128>(a, g, RW, st);
        return;
      }
      if (conv3_rw(a, 128) > 0) {
        dim3 g(a.B * a.Ho * a.Wo / 128, (a.Cout + 127) / 128, 1);
        // Chosen from ONE image's tile count (64 = the batch-8 grid's 512): the two forms walk
        // the channels in different chunk orders (CK), so a batch-size-driven choice made an
        // image's result depend on its batch (B = 16 vs 1 at the 32x32 level).
        // The 8-wave form as 4 x 2 waves of 32 x 64 (round 5: +0.3 % in the network against
        // 2 x 4 waves of 64 x 32, three interleaved pairs; 4 x 4 waves of 32 x 32 no better).
        if ((long)(a.Ho * a.Wo / 128) * g.y >= 64)
          conv3_launch<T, 128, 128, 2, 2, 64>(a, g, conv3_rw(a, 128), st);
        else
          conv3_launch<T, 128, 128, 4, 2, 128>(a, g, conv3_rw(a, 128), st);
        return;
      }
    }
  }
  if constexpr (V2) if (v2ok) {
    // Minimal epilogue when every tile lies inside one image (tile rows divide H*W, or the
    // per-image grid) and the tail is SiLU / none on 16-byte rows.
    constexpr int VEh = 16 / sizeof(T);
    const bool rows_ok = a.Cout % VEh == 0 && a.ldy % VEh == 0 && (!a.res1 || a.ldr1 % VEh == 0) &&
                         (!a.res2 || a.ldr2 % VEh == 0);
    const bool act_ok = a.act == ACT_NONE || a.act == ACT_SILU;
    const int HWo = a.Ho * a.Wo;
    auto minimal = [&](int BMv) { return rows_ok && act_ok && (batched || HWo % BMv == 0); };
#define DAC_V2(BM_, BN_, WGM_, WGN_, ST_, THR_)                                                   \
    {                                                                                            \
      dim3 g((Mg + BM_ - 1) / BM_, (a.Cout + BN_ - 1) / BN_, gz);                                \
      if (minimal(BM_))                                                                          \
        conv2_kernel<T, BM_, BN_, WGM_, WGN_, ST_, KH, KW, S, P, EPI_MIN><<<g, THR_, 0, st>>>(a); \
      else                                                                                       \
        conv2_kernel<T, BM_, BN_, WGM_, WGN_, ST_, KH, KW, S, P, EPI_ALL><<<g, THR_, 0, st>>>(a); \
      return;                                                                                    \
    }
    if constexpr (KH == 1) if (a.ln_g) {
      // Row-LayerNorm epilogue: one N tile must cover Cout exactly.
      if constexpr (sizeof(T) == 2)
        if (minimal(256) && a.Cout == 64 && !a.ss && a.act == ACT_NONE && !a.res2 && !a.bbias) {
          // One wave owns all 64 channels of its rows: the LN runs in registers.
          dim3 g((Mg + 255) / 256, 1, gz);
          conv2_kernel<T, 256, 64, 4, 1, 2, KH, KW, S, P, EPI_SWAP | EPI_LN><<<g, 256, 0, st>>>(a);
          return;
        }
      if (minimal(256) && a.Cout == 64) {
        dim3 g((Mg + 255) / 256, 1, gz);
        conv2_kernel<T, 256, 64, 4, 2, 3, KH, KW, S, P, EPI_LN><<<g, 512, 0, st>>>(a);
        return;
      }
      if (minimal(128) && a.Cout == 128) {
        dim3 g((Mg + 127) / 128, 1, gz);
        conv2_kernel<T, 128, 128, 2, 2, 2, KH, KW, S, P, EPI_LN><<<g, 256, 0, st>>>(a);
        return;
      }
      throw std::logic_error("conv: shape the engine never requests");
    }
    if constexpr (KH == 1) if (a.gna_stats) {
      // Input GroupNorm in the A path (conv_gna_ok mirrors this choice).
      if constexpr (sizeof(T) == 2)
        if (minimal(64) && a.Cout % 128 == 0 && !batched) {
          dim3 g((Mg + 63) / 64, a.Cout / 128, gz);
          conv2_kernel<T, 64, 128, 2, 2, 2, KH, KW, S, P, EPI_SWAP | EPI_GNA><<<g, 256, 0, st>>>(a);
          return;
        }
      throw std::logic_error("conv: conv_gna_ok promised an input-GroupNorm kernel");
    }
    if constexpr (KH == 1) if (a.lnf_cs) {
      // Input LayerNorm folded in (conv_lnf_ok mirrors these two choices).
      // (Swapped 64x128 tiles only. A 256x256 GEGLU | LNF tile existed in round 3; its fp16
      // outputs depended on the batch composition and it was slower than the unfolded chain, so
      // it was removed together with conv_lnf_ok's GEGLU case.)
      if constexpr (sizeof(T) == 2) {
        if (a.act != ACT_GEGLU && minimal(64) && a.Cout % 128 == 0) {
          dim3 g((Mg + 63) / 64, a.Cout / 128, gz);
          conv2_kernel<T, 64, 128, 2, 2, 2, KH, KW, S, P, EPI_SWAP | EPI_LNF><<<g, 256, 0, st>>>(a);
          return;
        }
      }
      throw std::logic_error("conv: conv_lnf_ok promised a folding kernel");
    }
    const int f2 = (KH == 1 && g_conv2_force32 > 0 && a.Ho > 1 && a.Wo > 1 && a.Ho * a.Wo <= 1024 && a.Ho * a.Wo >= 256 && a.ksplit <= 1 && a.act != ACT_GEGLU) ? g_conv2_force32 : g_conv2_force;
    if constexpr (KH == 1) if (f2 > 0) {
      switch (f2) {
        case 1: DAC_V2(256, 128, 4, 2, 3, 512)
        case 2: DAC_V2(128, 128, 2, 2, 2, 256)
        case 3: DAC_V2(256, 128, 4, 2, 2, 512)
        case 4: DAC_V2(128, 128, 2, 2, 3, 256)
        case 5: {
          dim3 g((Mg + 255) / 256, (a.Cout + 255) / 256, gz);
          conv2_kernel<T, 256, 256, 4, 2, 2, KH, KW, S, P, EPI_MIN><<<g, 512, 0, st>>>(a);
          return;
        }
        case 6: DAC_V2(128, 256, 2, 4, 2, 512)
        case 7: DAC_V2(128, 64, 2, 2, 2, 256)
        case 8: DAC_V2(64, 128, 2, 2, 2, 256)
        case 9: DAC_V2(64, 64, 2, 2, 3, 256)
        case 10: DAC_V2(128, 64, 2, 2, 3, 256)
        case 11: DAC_V2(64, 128, 2, 2, 3, 256)
        case 12: DAC_V2(64, 128, 2, 2, 4, 256)
        case 13:
          if constexpr (sizeof(T) == 2)
            if (minimal(64) && a.Cout % 128 == 0) {
              dim3 g((Mg + 63) / 64, a.Cout / 128, gz);
              conv2_kernel<T, 64, 128, 2, 2, 3, KH, KW, S, P, EPI_SWAP><<<g, 256, 0, st>>>(a);
              return;
            }
          DAC_V2(64, 128, 2, 2, 3, 256)
        case 17:
        case 18:
        case 19:
          if constexpr (sizeof(T) == 2)
            if (minimal(128) && a.Cout % 128 == 0) {
              // Deep rings (in-flight depth probe): 64x128 x 6 stages, 128x128 x 4 / 5 stages.
              if (f2 == 17) conv2_kernel<T, 64, 128, 2, 2, 6, KH, KW, S, P, EPI_SWAP><<<dim3((Mg + 63) / 64, a.Cout / 128, gz), 256, 0, st>>>(a);
              else if (f2 == 18) conv2_kernel<T, 128, 128, 2, 2, 4, KH, KW, S, P, EPI_SWAP><<<dim3((Mg + 127) / 128, a.Cout / 128, gz), 256, 0, st>>>(a);
              else conv2_kernel<T, 128, 128, 2, 2, 5, KH, KW, S, P, EPI_SWAP><<<dim3((Mg + 127) / 128, a.Cout / 128, gz), 256, 0, st>>>(a);
              return;
            }
          DAC_V2(64, 128, 2, 2, 2, 256)
        case 14:
        case 15:
        case 16:
          if constexpr (sizeof(T) == 2)
            if (minimal(128) && a.Cout % 128 == 0) {
              dim3 g((Mg + 127) / 128, a.Cout / 128, gz);
              if (f2 == 14) conv2_kernel<T, 128, 128, 2, 2, 2, KH, KW, S, P, EPI_SWAP><<<g, 256, 0, st>>>(a);
              else if (f2 == 15) conv2_kernel<T, 128, 128, 2, 2, 3, KH, KW, S, P, EPI_SWAP><<<g, 256, 0, st>>>(a);
              else conv2_kernel<T, 64, 128, 2, 2, 4, KH, KW, S, P, EPI_SWAP><<<dim3((Mg + 63) / 64, a.Cout / 128, gz), 256, 0, st>>>(a);
              return;
            }
          DAC_V2(64, 128, 2, 2, 2, 256)
        default: break;
      }
    }
    if constexpr (KH == 1) if (a.ksplit > 1 && a.part) {
      // Split-K (conv_split_ok): 64x128 tiles, grid z = ksplit, then the reduce + epilogue pass.
      if (a.ln_g || a.lnf_cs || a.gna_stats || batched || a.act == ACT_GEGLU)
        throw std::logic_error("conv: epilogue feature without a kernel for this shape");
      dim3 g((Mg + 63) / 64, (a.Cout + 127) / 128, a.ksplit);
      conv2_kernel<T, 64, 128, 2, 2, 2, KH, KW, S, P, EPI_PART><<<g, 256, 0, st>>>(a);
      conv_part_reduce<T>(a, st);
      return;
    }
    if constexpr (KH == 1) if (a.K <= BKE) {
      // One K tile (1x1 over 64 bf16 channels): no pipeline to fill, so a single small
      // stage (128x64, 4 waves) keeps several blocks resident per CU and their load
      // latencies overlap (measured best of 256x128 x {1,2,3} stages, 128x128, 128x64).
      DAC_V2(128, 64, 2, 2, 1, 256)
    }
    if constexpr (KH == 1) if (a.Cout <= 64) DAC_V2(128, 64, 2, 2, 2, 256)
    if (a.Cout <= 64) DAC_V2(256, 64, 4, 2, 3, 512)
    if constexpr (KH == 1) {
      // 1x1 / linear GEMMs (measured, tools/convbench 1x1 sweep): Cout <= 64 (K > 64) 128x64
      // with 2 stages (above); GEGLU projections 128x256 (8 waves of 64x64, 2 stages); wide
      // plain outputs 256x256 (8 waves of 64x128, 2 stages, minimal epilogue only: the
      // general one spills at this tile); the rest 64x128 with 2 stages (4 waves of 32x64),
      // which doubles the blocks of the small 32x32-level GEMMs over 128x128.
      if (a.act == ACT_GEGLU) {
        // Swapped tiles with the register GEGLU epilogue (weights in the w_gs order): no LDS
        // staging of the fp32 tile, 16-byte stores straight from the accumulators.
        if constexpr (sizeof(T) == 2)
          if (a.w_gs && a.b_gs && rows_ok && !a.res1 && !a.res2 && !a.bbias && !a.ss && g_geglu_sw > 0) {
            ConvArgs q = a;
            q.w = a.w_gs; q.bias = a.b_gs;
            const int cfg = g_conv2_force >= 20 && g_conv2_force <= 23 ? g_conv2_force - 19 : g_geglu_sw;
            if (cfg == 1 && (batched || HWo % 256 == 0) && a.Cout % 256 == 0) {
              conv2_kernel<T, 256, 256, 4, 4, 2, KH, KW, S, P, EPI_SWAP | EPI_GEGLU><<<dim3((Mg + 255) / 256, a.Cout / 256, gz), 1024, 0, st>>>(q);
              return;
            }
            if (cfg == 2 && (batched || HWo % 128 == 0) && a.Cout % 256 == 0) {
              conv2_kernel<T, 128, 256, 2, 4, 2, KH, KW, S, P, EPI_SWAP | EPI_GEGLU><<<dim3((Mg + 127) / 128, a.Cout / 256, gz), 512, 0, st>>>(q);
              return;
            }
            if (cfg == 3 && (batched || HWo % 256 == 0) && a.Cout % 128 == 0) {
              conv2_kernel<T, 256, 128, 4, 2, 2, KH, KW, S, P, EPI_SWAP | EPI_GEGLU><<<dim3((Mg + 255) / 256, a.Cout / 128, gz), 512, 0, st>>>(q);
              return;
            }
            if (cfg == 4 && (batched || HWo % 128 == 0) && a.Cout % 128 == 0) {
              conv2_kernel<T, 128, 128, 2, 2, 2, KH, KW, S, P, EPI_SWAP | EPI_GEGLU><<<dim3((Mg + 127) / 128, a.Cout / 128, gz), 256, 0, st>>>(q);
              return;
            }
          }
        // 256x256 tiles when they stay inside one image: half the LDS-DMA bytes per MFMA of
        // the 128x256 tiles, whose per-stage refill the MFMAs could not cover.
        if constexpr (sizeof(T) == 2)
          if (rows_ok && !a.res1 && !a.res2 && !a.bbias && (batched || HWo % 256 == 0) && a.Cout % 256 == 0 &&
              g_conv2_force == 0) {
            dim3 g((Mg + 255) / 256, a.Cout / 256, gz);
            conv2_kernel<T, 256, 256, 4, 2, 2, KH, KW, S, P, EPI_GEGLU><<<g, 512, 0, st>>>(a);
            return;
          }
        DAC_V2(128, 256, 2, 4, 2, 512)
      }
      if (a.Cout >= 1024 && minimal(256)) {
        dim3 g((Mg + 255) / 256, (a.Cout + 255) / 256, gz);
        conv2_kernel<T, 256, 256, 4, 2, 2, KH, KW, S, P, EPI_MIN><<<g, 512, 0, st>>>(a);
        return;
      }
      // bf16, whole tiles in one image, Cout a multiple of the tile: swapped operands +
      // register epilogue (no LDS round trip).
      if constexpr (sizeof(T) == 2)
        if (minimal(64) && a.Cout % 128 == 0 && g_conv2_force == 0) {
          dim3 g((Mg + 63) / 64, a.Cout / 128, gz);
          conv2_kernel<T, 64, 128, 2, 2, 2, KH, KW, S, P, EPI_SWAP><<<g, 256, 0, st>>>(a);
          return;
        }
      DAC_V2(64, 128, 2, 2, 2, 256)
    }
    if ((long)((Mg + 255) / 256) * ((a.Cout + 127) / 128) * gz >= 256) DAC_V2(256, 128, 4, 2, 3, 512)
    DAC_V2(128, 128, 2, 2, 3, 256)
#undef DAC_V2
  }
  if (a.Cout <= 16 && a.act != ACT_GEGLU) {
    dim3 g((Mg + 255) / 256, (a.Cout + 15) / 16, gz);
    conv_kernel<T, 256, 16, 4, 1, KH, KW, S, P><<<g, 256, 0, st>>>(a);
  } else if (a.Cout <= 64) {
    dim3 g((Mg + 255) / 256, (a.Cout + 63) / 64, gz);
    conv_kernel<T, 256, 64, 4, 1, KH, KW, S, P><<<g, 256, 0, st>>>(a);
  } else {
    dim3 g((Mg + 127) / 128, (a.Cout + 127) / 128, gz);
    conv_kernel<T, 128, 128, 2, 2, KH, KW, S, P><<<g, 256, 0, st>>>(a);
  }
}


}  // namespace dac
