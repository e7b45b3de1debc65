// conv3q.hip — fp8 ResBlock block2 (3x3, 64 -> 64) over an e4m3 input: the fp8 handles' MX path
// (BASELINE configs[4]) for the ResBlocks of the 256x256 and 128x128 levels
// (module_util.py:143-153: block2(SiLU(block1(x) * (1 + scale) + shift)) + res). Block1's epilogue
// writes h as e4m3 bytes with one E8M0 exponent per (pixel, 32-channel half) (conv_impl.h
// q8_store); this kernel DMAs those bytes straight into LDS (half the bytes of the 16-bit halo,
// all 64 channels in one 64-byte row) and runs the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4, twice the 16-bit MFMA rate per clock.
//
// Structure: conv3w_kernel's (weight-stationary, 8 waves, each with a private 2-stage ring of
// 64-pixel row segments, persistent XCD bands, swapped operands + register epilogue), with
// three stages per segment (one per kernel row kh) instead of six.
//
// K arrangement of one 16x16x128 MFMA = two taps of one kernel row: lane (r, g) supplies 32
// bytes, the first 16 holding channels 16g..16g+15 of tap A, the second 16 the same channels of
// tap B. The hardware reads them as k slots 16g.. and 64 + 16g.. (measured, conv8.hip), so the
// 32-slot scale blocks are {tap A ch 0-31, tap A ch 32-63, tap B ch 0-31, tap B ch 32-63} and lane
// group g supplies the exponent of block g: (g < 2 ? tap A : tap B, half g & 1). A kernel row's
// taps pair as (kw0 | kw1) and (kw2 | zero weights): 6 MFMAs per 16x16 output tile against 18
// 16-bit ones (1.5x fewer MFMA cycles). The pixel operand of pair (kw, kw + 1) for tile i is
// {F[i + kw], F[i + kw + 1]} where F[f] is conv3w's halo fragment (lane (r, g): halo pixel
// TM * r + f, 16-byte slot g), so a stage still reads only TM + 2 fragments.
#include "conv_impl.h"

namespace dac {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int C3Q_WAVES = 8, C3Q_TM = 4, C3Q_SEG = 16 * C3Q_TM;
constexpr int C3Q_NI = (C3Q_SEG + 2 + 15) / 16;          // halo DMA instructions per stage
constexpr int C3Q_STAGE = C3Q_NI * 1024 + 256;           // + one 4-byte-per-lane exponent DMA
constexpr int C3Q_WBYTES = 9 * 64 * 64;                  // e4m3 weights: 9 taps x 64 rows x 64 B
constexpr int C3Q_SMEM = C3Q_WBYTES + C3Q_WAVES * 2 * C3Q_STAGE + 256;   // + the bias
static_assert(C3Q_SMEM <= 160 * 1024, "LDS");

DEV void buf_lds4(const void* base, int nbytes, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes, 0x00020000), (lds_void_t*)lds, 4,
      voff, soff, 0, 0);
}
DEV void mma8(f32x4& acc, const i32x8& w, const i32x8& x, int sw, int sx) {
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w, x, acc, 0, 0, 0, sw, 0, sx);
}

template <typename T>
__global__ void __launch_bounds__(64 * C3Q_WAVES)
conv3q_kernel(ConvArgs a, const uint8_t* __restrict__ q8w, const uint8_t* __restrict__ q8s, int ntiles, int delay) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int NWV = C3Q_WAVES, TM = C3Q_TM, NF = TM + 2, SEG = C3Q_SEG, NI = C3Q_NI, STAGE = C3Q_STAGE;
  using SA = RowSwz<4, TM>;
  using SB = RowSwz<4, 1>;
  __shared__ __attribute__((aligned(1024))) char smem[C3Q_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;

  // Weights -> LDS, once: DMA instruction q fills tap region q >> 2 (4 KB), physical rows
  // (q & 3) * 16 + lane / 4, 16-byte slot lane & 3; MFMA row p holds output channel wperm64(p).
  for (int q = wave; q < 36; q += NWV) {
    const int tap = q >> 2, rho = (q & 3) * 16 + (lane >> 2);
    const uint8_t* src = q8w + (size_t)wperm64(rho) * 576 + tap * 64 + SB::slot(rho, lane & 3) * 16;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(smem + q * 1024), 16, 0, 0);
  }
  // Weight exponents of this lane's rows (block g: tap kw = g >> 1 of the pair, half g & 1),
  // one byte per kernel row kh: pair (kw0 | kw1) in ws0, pair (kw2 | zero) in ws1.
  uint32_t ws0[4], ws1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint8_t* s = q8s + wperm64(16 * j + lr) * 18 + (lg & 1);
    const int kwA = lg >> 1;
    ws0[j] = s[2 * kwA] | (uint32_t)s[2 * (3 + kwA)] << 8 | (uint32_t)s[2 * (6 + kwA)] << 16;
    ws1[j] = lg < 2 ? (s[4] | (uint32_t)s[10] << 8 | (uint32_t)s[16] << 16) : 0x7f7f7fu;
  }
  // The bias waits in LDS for the epilogues (16 registers fewer across the main loop).
  if (tid < 64) reinterpret_cast<float*>(smem + C3Q_SMEM - 256)[tid] = a.bias ? a.bias[tid] : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int xcd = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int t_end = (int)((long)(xcd + 1) * ntiles / 8);
  const int stride = nbx * NWV;
  int t = (int)((long)xcd * ntiles / 8) + (blockIdx.x >> 3) * NWV + wave;
  if (t >= t_end) return;

  char* ring = smem + C3Q_WBYTES + wave * 2 * STAGE;
  const char* wl = smem;
  const int segs = a.Wo / SEG;
  constexpr unsigned OOB = 0x80000000u;
  // Halo DMA: instruction j fills physical rows j * 16 + lane / 4 = logical halo row dr[j]
  // (pixel ow0 - 1 + dr of the kernel row), logical slot SA::slot at physical slot lane & 3.
  int dr[NI], boffs[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int R = SA::logical(j * 16 + (lane >> 2));
    dr[j] = R;
    boffs[j] = R < SEG + 2 ? R * a.ld1 + SA::slot(R, lane & 3) * 16 : (int)OOB;
  }
  int aoff[NF + 1], boff[4];
#pragma unroll
  for (int f = 0; f <= NF; ++f) aoff[f] = SA::phys(TM * lr + f) * 64 + (SA::slot(TM * lr + f, lg) << 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) boff[j] = (16 * j + lr) * 64 + (SB::slot(16 * j + lr, lg) << 4);
  const int npix = a.B * a.Hs * a.Ws;
  const char* xbase = reinterpret_cast<const char*>(a.x1) - a.ld1;       // pixel before the row
  const int x_bytes = npix * a.ld1 + a.ld1;
  // Exponent DMA: lane l's dword = halo pixels 2l - 1, 2l (2 bytes each) counted from the
  // segment's first halo pixel; the base sits 4 bytes before xs8 so offsets stay positive. The
  // left-padding pixel's exponent lane reads nothing (its data is zero; a 0 exponent is finite).
  const char* sbase = reinterpret_cast<const char*>(a.xs8) - 4;
  const int s_bytes = 2 * npix + 4;

  auto issue = [&](int tt, int kh, int slot) {
    const bool live = tt < t_end;
    const int rr = live ? tt / segs : 0, ow0 = live ? (tt - rr * segs) * SEG : 0;
    const int b = rr / a.Ho, oh = rr - b * a.Ho;
    const int ih = oh + kh - 1;
    const bool row_ok = live && (unsigned)ih < (unsigned)a.Hs;
    const int pix0 = (b * a.Hs + ih) * a.Ws + ow0;
    const int soff = row_ok ? pix0 * a.ld1 : 0;
    const bool lpad = ow0 == 0, rpad = ow0 + SEG == a.Wo;
    char* dst = ring + slot * STAGE;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int vo = row_ok ? boffs[j] : (int)OOB;
      if (j == 0) vo = (lpad && dr[j] == 0) ? (int)OOB : vo;
      if ((SEG + 1) / 16 == j) vo = (rpad && dr[j] == SEG + 1) ? (int)OOB : vo;
      buf_lds16(xbase, x_bytes, dst + j * 1024, vo, soff);
    }
    buf_lds4(sbase, s_bytes, dst + NI * 1024, (row_ok && !(lpad && lane == 0)) ? lane * 4 : (int)OOB,
             row_ok ? 2 * pix0 : 0);
  };

  const int nb = 16 * lg;
  const float* sbias = reinterpret_cast<const float*>(smem + C3Q_SMEM - 256);
  // This lane's exponent bytes: pair q, tile i needs halo pixel f = i + 2q + (g >= 2), half g & 1,
  // at stage byte 2 + 2f + (g & 1) = 2 (i + 2q) + sh0 from 8 * lr. Shifting the lane's 16 bytes
  // right by sh0 puts k = i + 2q at byte 2k.
  const int sh0 = 2 + ((lg >> 1) << 1) + (lg & 1);
  const bool shw = sh0 >= 4;
  const uint32_t shb = (uint32_t)(sh0 & 3);

  if (NWV > 4 && (wave & 4))
    for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(8);
  issue(t, 0, 0);
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
    for (int kh = 0; kh < 3; ++kh, ++g) {
      // Own DMA of this stage landed (at a tile's first stage the previous epilogue's 2 * TM
      // stores, issued after it, may stay in flight).
      if (kh == 0 && g > 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(2 * TM) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if (kh == 2) epi_prefetch<T, TM>(a, nb, b, [&](int i) { return (size_t)m0 + TM * lr + i; }, pref);
      issue(kh == 2 ? tn : t, (kh + 1) % 3, slot ^ 1);

      const char* st = ring + slot * STAGE;
      // Operand tuples loaded in place (no register copies into the 8-VGPR MFMA operands):
      // pixel tuple f = {F[f], F[f + 1]} serves pair (kw0 | kw1) of tile f and pair
      // (kw2 | zero) of tile f - 2 (its second half then meets zero weights; F[TM + 2] is a
      // halo row past the segment, finite: data or the DMA's zero fill).
      i32x8 xb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        xb[f].lo = *reinterpret_cast<const i32x4*>(st + aoff[f]);
        xb[f].hi = *reinterpret_cast<const i32x4*>(st + aoff[f + 1]);
      }
      const uint64_t e01 = *reinterpret_cast<const uint64_t*>(st + NI * 1024 + 8 * lr);
      const uint64_t e23 = *reinterpret_cast<const uint64_t*>(st + NI * 1024 + 8 * lr + 8);
      const char* wr = wl + kh * 3 * 4096;
      i32x8 wa[4], wb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wa[j].lo = *reinterpret_cast<const i32x4*>(wr + boff[j]);
        wa[j].hi = *reinterpret_cast<const i32x4*>(wr + 4096 + boff[j]);
        wb[j].lo = *reinterpret_cast<const i32x4*>(wr + 8192 + boff[j]);
        wb[j].hi = i32x4{0, 0, 0, 0};
      }
      const uint32_t d0 = (uint32_t)e01, d1 = (uint32_t)(e01 >> 32), d2 = (uint32_t)e23, d3 = (uint32_t)(e23 >> 32);
      const uint32_t s0 = shw ? d1 : d0, s1 = shw ? d2 : d1, s2 = shw ? d3 : d2, s3 = shw ? 0u : d3;
      uint32_t X[6];
      X[0] = __builtin_amdgcn_alignbyte(s1, s0, shb);
      X[2] = __builtin_amdgcn_alignbyte(s2, s1, shb);
      X[4] = __builtin_amdgcn_alignbyte(s3, s2, shb);
      X[1] = X[0] >> 16;
      X[3] = X[2] >> 16;
      X[5] = X[4] >> 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int sw = (int)(ws0[j] >> (8 * kh));
#pragma unroll
        for (int i = 0; i < TM; ++i) mma8(acc[i][j], wa[j], xb[i], sw, (int)X[i]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int sw = (int)(ws1[j] >> (8 * kh));
#pragma unroll
        for (int i = 0; i < TM; ++i) mma8(acc[i][j], wb[j], xb[i + 2], sw, (int)X[i + 2]);
      }
      // Pin this stage's MFMAs before the next stage's wait: they read only registers, so the
      // compiler would otherwise sink all three stages' MFMAs below the last stage's loads (and
      // spill the operands of all of them).
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(acc[i][j]));
      slot ^= 1;
    }
    // The prefetched epilogue operands are older than the next stage's NI + 1 DMA instructions.
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI + 1) : "memory");
    float bi[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bi[e] = sbias[nb + e];
    epi_regs16<T, TM, false, true>(a, acc, bi, nb, b, [&](int i) { return (size_t)m0 + TM * lr + i; }, &pref);
    if (tn >= t_end) break;
    t = tn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool conv3q_ok(const ConvArgs& a) {
  return a.xs8 && !a.x2 && a.Cin == 64 && a.C1 >= 64 && a.Cout == 64 && a.K == 576 && a.ld1 == 64 && !a.up &&
         a.Ho == a.Hs && a.Wo == a.Ws && a.Wo % C3Q_SEG == 0 && a.zero && a.amode == 0 && a.w_bstride == 0 &&
         !a.ln_g && !a.lnf_cs && !a.gna_stats && !a.y2 && !a.ys8 && a.cwrap == 0 &&
         (a.act == ACT_NONE || a.act == ACT_SILU) && a.ldy % 8 == 0 && (!a.res1 || a.ldr1 % 8 == 0) && !a.res2 &&
         !a.bbias && !(a.ss && a.res1) && (!a.ss || (a.ss_ld % 4 == 0 && ((uintptr_t)a.ss & 15) == 0)) &&
         (size_t)a.B * a.Hs * a.Ws * 64 + 64 < ((size_t)1 << 31);
}

template <typename T>
void conv3q(const ConvArgs& a, const uint8_t* q8w, const uint8_t* q8s, hipStream_t st) {
  if (!conv3q_ok(a) || !q8w || !q8s) throw std::invalid_argument("conv3q: arguments rejected by conv3q_ok");
  const int ntiles = a.B * a.Ho * (a.Wo / C3Q_SEG);
  conv3q_kernel<T><<<conv3w_blocks(ntiles, C3Q_WAVES), 64 * C3Q_WAVES, 0, st>>>(a, q8w, q8s, ntiles, 6);
}
template void conv3q<bf16>(const ConvArgs&, const uint8_t*, const uint8_t*, hipStream_t);
template void conv3q<f16>(const ConvArgs&, const uint8_t*, const uint8_t*, hipStream_t);

}  // namespace dac
