// conv_edge.hip — the two edge convs of the ConditionalUNet for 16-bit (bf16 / f16) handles, each a
// dedicated kernel because the generic implicit GEMM wastes most of its work on them:
// (1) init_conv (conv7_kernel) and (2) final_conv (conv3n_kernel, below).
//
// (1) init_conv: 7x7, stride 1, pad 3, Cin = 8 ([xt | mu], 6 real channels padded to one 16-byte vector), Cout = 64, no bias/act
// (DenoisingUNet_arch.py:50 `default_conv(in_nc*2, nf, 7)`, module_util.py:111-112).
//
// Why a kernel of its own: as a generic implicit GEMM the layer has K = 7 rows x 8 taps x 8
// channels (x2 for the split-precision hi|lo weights), and every 64-element K tile re-reads
// 8 neighbouring input pixels per output pixel (8x im2col redundancy through LDS-DMA), which
// ran at ~150 TF/s (135 us per 256^2 x 8 launch).
//
// Here:
//  * Weight-stationary in VGPRs: wave w owns output channels 16w..16w+15 and keeps their whole
//    K (14 chunks x {hi, lo} = 28 MFMA A fragments, 112 VGPRs) for the kernel's lifetime.
//  * The K chunk c = 2*kh + h covers taps 4h..4h+3 of kernel row kh; MFMA lane group g supplies
//    tap 4h+g, channels 0..7 = one 16-byte pixel. So the B operand of pixel j is simply the
//    halo pixel j + 4h + g of input row kh, read straight from LDS with one ds_read_b128 —
//    the input row band (7 rows x 264 pixels x 16 B) lands in LDS once per tile and every
//    tap reads a shifted window of it. Tap 7 gets zero weights (the halo is finite).
//  * Persistent blocks walk row-segment tiles (256 output pixels of one image row), each XCD a
//    contiguous band of rows so neighbouring tiles' shared input rows hit the same L2. The next
//    tile's halo is DMA'd (global_load_lds) into the other LDS buffer under this tile's MFMAs;
//    one barrier per tile.
//  * Epilogue from registers: lane (r, g) of pixel tile t holds channels 16w + 4g .. +3 of
//    pixel 16t + r: one 8-byte store, bias (if any) added in fp32.
// MFMA: 16x16x32 bf16 / f16, A = weights (rows = output channels), B = pixels; hi and lo parts
// accumulate into the same fp32 accumulator (= W.x with ~2^-17 weight error).
#include "common.h"
#include "kernels.h"

namespace dac {

typedef __attribute__((address_space(3))) void lds7_t;
typedef __attribute__((address_space(1))) const void gbl7_t;

constexpr int C7_SEG = 256;                       // output pixels per tile
constexpr int C7_HP = C7_SEG + 8;                 // halo pixels per input row (ow0-3 .. ow0+260)
constexpr int C7_ITEMS = 7 * C7_HP;               // 16-byte halo items per tile
constexpr int C7_INSTR = (C7_ITEMS + 63) / 64;    // LDS-DMA wave-instructions per tile (29)
constexpr int C7_BUF = C7_INSTR * 1024;           // bytes per halo buffer

bool conv7_ok(const ConvArgs& a) {
  const int np = a.cwrap ? 2 : 1;
  return a.Cin == 8 && a.ld1 == 8 && a.Cout == 64 && a.K == np * 7 * 8 * 8 && !a.x2 && !a.up && a.zero &&
         a.amode == 0 && a.w_bstride == 0 && !a.ss && a.act == ACT_NONE && !a.res1 && !a.res2 && !a.bbias &&
         !a.ln_g && a.ldy % 4 == 0 && a.Ho == a.Hs && a.Wo == a.Ws;
}

template <typename T, int NP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv7_kernel(ConvArgs a, int ntiles) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  __shared__ __attribute__((aligned(1024))) char smem[2 * C7_BUF];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int nseg = (a.Wo + C7_SEG - 1) / C7_SEG;

  // Weight fragments (row-tap layout [o][part][kh][8 taps][8 ch], engine.cpp Packer::conv_dual).
  const T* wg = reinterpret_cast<const T*>(a.w);
  const int o = 16 * wave + lr;
  u32x4 wf[14][NP];
#pragma unroll
  for (int c = 0; c < 14; ++c)
#pragma unroll
    for (int p = 0; p < NP; ++p)
      // Tap 7 (odd chunk, lane group 3) is the row padding: forced to zero here, so the
      // result never depends on what the packer left there.
      wf[c][p] = ((c & 1) && lg == 3)
                     ? u32x4{0u, 0u, 0u, 0u}
                     : *reinterpret_cast<const u32x4*>(wg + (size_t)o * NP * 448 + p * 448 + (c >> 1) * 64 +
                                                       ((c & 1) * 4 + lg) * 8);
  float bi[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bi[e] = a.bias ? a.bias[16 * wave + 4 * lg + e] : 0.f;

  // XCD-aware tile walk: XCD x (= blockIdx % 8) owns tiles [lo_x, hi_x); its k-th block takes
  // lo_x + k, lo_x + k + nbx, ... (nbx = blocks on that XCD).
  // (Grids that are not a multiple of 8 walk the tiles with a plain grid stride.)
  const int G = gridDim.x;
  int t0 = blockIdx.x, nbx = G, hi_x = ntiles;
  if ((G & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    nbx = G >> 3;
    t0 = (int)((long)ntiles * xcd / 8) + (blockIdx.x >> 3);
    hi_x = (int)((long)ntiles * (xcd + 1) / 8);
  }

  const char* zero = reinterpret_cast<const char*>(a.zero);
  const char* xs = reinterpret_cast<const char*>(a.x1);
  auto issue = [&](int t, int buf) {
    const int seg = t % nseg, row = t / nseg;          // row = b * Ho + oh
    const int b = row / a.Ho, oh = row - b * a.Ho;
    const int ow0 = seg * C7_SEG;
    char* dst = smem + buf * C7_BUF;
    for (int n = wave; n < C7_INSTR; n += 4) {
      const int i = n * 64 + lane;
      const char* src = zero;
      if (i < C7_ITEMS) {
        const int r = i / C7_HP, p = i - r * C7_HP;
        const int ih = oh - 3 + r, iw = ow0 - 3 + p;
        if ((unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws)
          src = xs + ((size_t)(b * a.Hs + ih) * a.Ws + iw) * 16;
      }
      __builtin_amdgcn_global_load_lds((gbl7_t*)src, (lds7_t*)(dst + n * 1024), 16, 0, 0);
    }
  };

  T* y = reinterpret_cast<T*>(a.y);
  int t = t0, buf = 0;
  if (t < hi_x) issue(t, 0);
  for (; t < hi_x; t += nbx, buf ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own halo DMA of tile t (and old stores)
    __builtin_amdgcn_s_barrier();                        // all halos in; tile t-1 fully read
    asm volatile("" ::: "memory");
    if (t + nbx < hi_x) issue(t + nbx, buf ^ 1);
    const char* hb = smem + buf * C7_BUF;
    const int seg = t % nseg, row = t / nseg;
    const int ow0 = seg * C7_SEG;
    T* yrow = y + (size_t)row * a.Wo * a.ldy + 16 * wave + 4 * lg;
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) {
      f32x4 acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 14; ++c) {
        const char* rb = hb + ((c >> 1) * C7_HP + grp * 128 + lr + (c & 1) * 4 + lg) * 16;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const u32x4 xf = *reinterpret_cast<const u32x4*>(rb + q * 256);
#pragma unroll
          for (int p = 0; p < NP; ++p) Mma<T>::run(acc[q], wf[c][p], xf);
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int ow = ow0 + grp * 128 + q * 16 + lr;
        if (ow < a.Wo) {
          typename Vec8<T>::t2 v0, v1;
          v0[0] = (T)(acc[q][0] + bi[0]); v0[1] = (T)(acc[q][1] + bi[1]);
          v1[0] = (T)(acc[q][2] + bi[2]); v1[1] = (T)(acc[q][3] + bi[3]);
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          u32x2 st;
          st[0] = __builtin_bit_cast(uint32_t, v0);
          st[1] = __builtin_bit_cast(uint32_t, v1);
          *reinterpret_cast<u32x2*>(yrow + (size_t)ow * a.ldy) = st;
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename T>
void conv7(const ConvArgs& a, hipStream_t st) {
  const int nseg = (a.Wo + C7_SEG - 1) / C7_SEG;
  const int ntiles = a.B * a.Ho * nseg;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  int G = 2 * ncu;                                 // two 4-wave blocks per CU (59 KB LDS each)
  if (G > ntiles) G = ntiles;
  if (G >= 8) G &= ~7;
  if (G < 1) return;
  if (a.cwrap) conv7_kernel<T, 2><<<G, 256, 0, st>>>(a, ntiles);
  else conv7_kernel<T, 1><<<G, 256, 0, st>>>(a, ntiles);
}

// ---------------------------------------------------------------------------------------
// (2) final_conv: 3x3, stride 1, pad 1, Cin = 64 -> Cout = out_nc (<= 4), + bias
// (DenoisingUNet_arch.py:112 `final_conv = nn.Conv2d(nf, out_nc, 3, 1, 1)`), with plain or
// split-precision weights. The generic path ran it as a 16-column GEMM over K = 9 x 128 (the
// hi|lo parts along K) at 55 us per 256^2 x 8 launch; the layer is a pure stream of its 67 MB
// input (8 us at HBM peak).
//  * The hi and lo weights are separate MFMA A rows (rows 0..3 hi, 4..7 lo of output channels
//    0..3), so K is 9 taps x 64 channels = 18 chunks of 32, all 18 A fragments resident in
//    VGPRs; the output channel c is row c + row c+4 = one xor-16 shuffle in the epilogue.
//  * A tile is 4 output rows x 64 pixels; its halo (6 input rows x 66 pixels x 128 B) is DMA'd
//    into LDS with the 16-byte slot XOR-swizzled by (halo pixel & 7) at the source, which keeps
//    every ds_read_b128 lane group on 16 distinct bank quads for any tap offset. (One-row tiles
//    re-read every input row 3x through the LDS-DMA path and ran at 1.7 TB/s.)
//  * One 4-wave block per CU, wave w owns pixel columns 16w..16w+15 of the tile's 4 rows (4
//    independent accumulator chains); a 3-slot ring keeps two tiles' halos loading while one is
//    consumed; persistent XCD-banded tile walk.
constexpr int CN_SEG = 64;                        // output pixels per tile row
constexpr int CN_R = 4;                           // output rows per tile
constexpr int CN_HP = CN_SEG + 2;                 // halo pixels per input row
constexpr int CN_PIX = (CN_R + 2) * CN_HP;        // 128-byte halo pixels per tile (396)
constexpr int CN_INSTR = 52;                      // LDS-DMA instructions per tile (>= 396/8), 13 per wave
constexpr int CN_SLOT = CN_INSTR * 1024;
constexpr int CN_ST = 3;                          // ring slots (156 KB)
static_assert(CN_INSTR * 8 >= CN_PIX && CN_INSTR % 4 == 0, "halo");

bool conv3n_ok(const ConvArgs& a) {
  const bool dual = a.Cin == 128 && a.x2 == a.x1 && a.ld2 == a.ld1 && a.C1 == 64 && a.cwrap == 0;
  const bool plain = a.Cin == 64 && a.C1 >= 64 && !a.x2;
  return (dual || plain) && a.K == 9 * a.Cin && a.Cout >= 1 && a.Cout <= 4 && a.ld1 % 8 == 0 && !a.up &&
         a.zero && a.amode == 0 && a.w_bstride == 0 && !a.ss && a.act == ACT_NONE && !a.res1 && !a.res2 &&
         !a.bbias && !a.ln_g && a.Ho == a.Hs && a.Wo == a.Ws && a.Wo % CN_SEG == 0 && a.Ho % CN_R == 0 &&
         a.ldy >= a.Cout;
}

template <typename T, int NP>
__global__ void __launch_bounds__(256) conv3n_kernel(ConvArgs a, int ntiles) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  __shared__ __attribute__((aligned(1024))) char smem[CN_ST * CN_SLOT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int nseg = a.Wo / CN_SEG, nrb = a.Ho / CN_R;

  // A fragments: row lr = output channel (lr & 3) of part lr >> 2 (0 hi, 1 lo); rows past the
  // parts / channels are zero. Weight layout [o][tap][part][64] (engine.cpp Packer::conv_dual).
  const T* wg = reinterpret_cast<const T*>(a.w);
  const int o = lr & 3, part = lr >> 2;
  const bool live = o < a.Cout && part < NP;
  u32x4 wf[18];
#pragma unroll
  for (int c = 0; c < 18; ++c) {
    const int tap = c >> 1, h = c & 1;
    wf[c] = live ? *reinterpret_cast<const u32x4*>(wg + ((size_t)o * 9 + tap) * 64 * NP + part * 64 + 32 * h + 8 * lg)
                 : u32x4{0u, 0u, 0u, 0u};
  }
  const float bias = (a.bias && lg < a.Cout) ? a.bias[lg] : 0.f;    // of the channel this lane stores

  const int G = gridDim.x;
  int t0 = blockIdx.x, nbx = G, hi_x = ntiles;
  if ((G & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    nbx = G >> 3;
    t0 = (int)((long)ntiles * xcd / 8) + (blockIdx.x >> 3);
    hi_x = (int)((long)ntiles * (xcd + 1) / 8);
  }
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const char* xs = reinterpret_cast<const char*>(a.x1);
  const size_t ldb = (size_t)a.ld1 * 2;
  // Tile t = ((b * nrb) + row block) * nseg + seg. Its halo -> ring slot; lane l of instruction
  // n fills halo pixel i = 8n + l/8, physical slot l&7 with logical slot (l&7) ^ (i&7). Every
  // wave issues exactly 13 instructions per tile (zero-page sources past the tile range).
  auto issue = [&](int t, int slot) {
    char* dst = smem + slot * CN_SLOT;
    const bool tv = t < hi_x;
    const int seg = t % nseg, rb = t / nseg;
    const int b = rb / nrb, oh0 = (rb - b * nrb) * CN_R;
#pragma unroll
    for (int k = 0; k < CN_INSTR / 4; ++k) {
      const int n = wave + 4 * k;
      const int i = 8 * n + (lane >> 3);
      const char* src = zero;
      if (tv && i < CN_PIX) {
        const int r = i / CN_HP, p = i - r * CN_HP;
        const int ih = oh0 - 1 + r, iw = seg * CN_SEG - 1 + p;
        if ((unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws)
          src = xs + ((size_t)(b * a.Hs + ih) * a.Ws + iw) * ldb + (((lane & 7) ^ (i & 7)) << 4);
      }
      __builtin_amdgcn_global_load_lds((gbl7_t*)src, (lds7_t*)(dst + n * 1024), 16, 0, 0);
    }
  };

  T* y = reinterpret_cast<T*>(a.y);
  constexpr int ND = CN_INSTR / 4;                // DMA instructions per wave per tile
  int t = t0;
#pragma unroll
  for (int s = 0; s < CN_ST - 1; ++s) issue(t + s * nbx, s);
  for (int it = 0; t < hi_x; t += nbx, ++it) {
    // Own DMA of tile t done. vmcnt is in issue order; younger than it: the next tile's ND DMAs
    // plus the CN_R stores of each iteration since (none, one, then two iterations' worth).
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(ND) : "memory");
    else if (it == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(ND + CN_R) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(ND + 2 * CN_R) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + (CN_ST - 1) * nbx, (it + CN_ST - 1) % CN_ST);   // the slot read at iteration it-1
    const char* hb = smem + (it % CN_ST) * CN_SLOT;
    f32x4 acc[CN_R];
#pragma unroll
    for (int q = 0; q < CN_R; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 18; ++c) {
      const int kh = (c >> 1) / 3, kw = (c >> 1) % 3, h = c & 1;
#pragma unroll
      for (int q = 0; q < CN_R; ++q) {
        const int i = (q + kh) * CN_HP + 16 * wave + lr + kw;
        const u32x4 xf = *reinterpret_cast<const u32x4*>(hb + i * 128 + (((4 * h + lg) ^ (i & 7)) << 4));
        Mma<T>::run(acc[q], wf[c], xf);
      }
    }
    const int seg = t % nseg, rb = t / nseg;
    const int ow = seg * CN_SEG + 16 * wave + lr;
#pragma unroll
    for (int q = 0; q < CN_R; ++q) {
      // lane (lr, g) holds rows 4g..4g+3 of pixel lr: g = 0 the hi rows, g = 1 the lo rows.
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = NP == 2 ? red16_sum(acc[q][e]) : acc[q][e];
      // Lane (lr, g) stores channel g of pixel lr (one 2-byte store instruction per wave and
      // row; with ldy >= 4 the padding channels Cout..3 are written as 0).
      float mine = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float ve = __shfl(v[e], lr, 64);
        if (lg == e) mine = ve;
      }
      const size_t m = ((size_t)rb * CN_R + q) * a.Wo + ow;     // (b*Ho + oh0 + q) * Wo + ow
      if (lg < a.ldy) y[m * a.ldy + lg] = (T)(lg < a.Cout ? mine + bias : 0.f);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename T>
void conv3n(const ConvArgs& a, hipStream_t st) {
  const int ntiles = a.B * (a.Ho / CN_R) * (a.Wo / CN_SEG);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  int G = ncu;                                     // one 4-wave block per CU (156 KB ring)
  if (G > ntiles) G = ntiles;
  if (G >= 8) G &= ~7;
  if (G < 1) return;
  if (a.Cin == 128) conv3n_kernel<T, 2><<<G, 256, 0, st>>>(a, ntiles);
  else conv3n_kernel<T, 1><<<G, 256, 0, st>>>(a, ntiles);
}

template void conv7<bf16>(const ConvArgs&, hipStream_t);
template void conv7<f16>(const ConvArgs&, hipStream_t);
template void conv3n<bf16>(const ConvArgs&, hipStream_t);
template void conv3n<f16>(const ConvArgs&, hipStream_t);

}  // namespace dac
