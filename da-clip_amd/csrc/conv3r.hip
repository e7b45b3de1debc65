// conv3r.hip — register-stationary 3x3 conv, 64 -> 64 channels (16-bit types): the UNet's
// 64-channel ResBlock convs and the last up level's default_conv on rows of >= 256 pixels
// (module_util.py:111-153, DenoisingUNet_arch.py:96; the 256x256 level at nf = 64: 8 launches per
// UNet step — 2 block1 with scale/shift + SiLU, 5 block2 with SiLU + residual, 1 plain).
//
// Why a new form: the LDS-resident-weight kernels (v4, v5) read every MFMA's weight operand from
// LDS and re-stage the halo per kernel row, and a stage's DMA, barrier and epilogue sit on each
// wave's critical path (v5: MFMA busy 26 %). Here each wave keeps its whole weight
// slice in VGPRs for the kernel's lifetime — 32 output channels x K = 576 (9 taps x 64 channels)
// = 36 A fragments, 144 VGPRs — and LDS carries only the input rows:
//   * a block (4 waves, 2 blocks per CU) owns a 128-pixel-wide strip of one image over RB output
//     rows (a "band"); wave (g, h) computes pixels 64 g .. 64 g + 63 of each row for output
//     channels 32 h .. 32 h + 31;
//   * the strip's input rows (130 halo pixels x 64 channels, 17 KB) stream through a 4-slot LDS
//     ring by buffer-descriptor LDS-DMA, ONE new row per output row (the two rows above stay
//     resident), issued a full row step ahead; one barrier per output row;
//   * per (kernel row, 32-channel chunk) a wave reads 6 B fragments (v4's interleaved-pixel
//     trick: lane row m of tile i is pixel 4 m + i, so tap kw of tile i is fragment i + kw) for
//     24 MFMAs, i.e. one 1 KB LDS read per 4 MFMAs: ~25 % of the LDS port at full MFMA rate;
//   * the epilogue (bias, per-image scale / shift, SiLU, residual) holds 8 channels of one pixel
//     per lane and tile -> 16-byte loads and stores; its folded per-channel terms sit in LDS, and
//     block2's residual rows are requested at the row start so they land under the MFMAs.
// Two details decide the speed (measured): every wait the compiler would put in the
// row loop for the prologue's weight loads is hoisted out (a counted vmcnt there waits for the
// row's fresh DMA every row), and the kernel must stay at <= 256 VGPRs with no spill (a spilled
// weight fragment reloads through scratch, i.e. another vmcnt on the DMA). 128-pixel rows (the
// 128x128 level) keep v5: with two rows per band there, the per-block weight load dominates.
// LDS image of an input row: halo pixel p (input column x0 - 1 + p) at physical slot
// P = p ^ ((p >> 2) & 1), its 16-byte channel chunk q at chunk q ^ ((P >> 2) & 7): every
// ds_read_b128 lane group of the B-fragment reads hits 16 distinct bank quads (exhaustive check
// over fragments, chunks and pixel groups). The DMA stays lane-linear (lane l fills slot
// 8 j + l / 8, chunk l % 8) with the permutation applied on the source side.
// Results do not depend on the band height RB or on the batch: every output is the same
// ordered sum (kernel row, chunk, tap) in the MFMA and the same epilogue, whatever block owns it.
#include "conv_impl.h"

namespace dac {

namespace {
constexpr unsigned C3R_OOB = 0x80000000u;
constexpr int C3R_SLOTS = 4;

DEV int c3r_phys(int p) { return p ^ ((p >> 2) & 1); }          // an involution
DEV int c3r_chunk(int P, int q) { return q ^ ((P >> 2) & 7); }   // logical <-> physical chunk

// Four output values of one pixel as one 8-byte store (the CIN 128 form's 16-row tiles).
template <typename T> DEV void store4(T* p, const float* v) {
  typedef T T4 __attribute__((ext_vector_type(4)));
  T4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (T)v[e];
  *reinterpret_cast<T4*>(p) = o;
}

// Geometry per input width: CIN = 64 (one 64-channel source half) or 128 (two halves: the
// up path's torch.cat of two 64-channel tensors, DenoisingUNet_arch.py:158-161, or one
// 128-channel tensor). A block is 4 waves over SW output pixels x 64 output channels:
//   CIN 64 : 2 pixel groups of 64 x 2 channel halves of 32 (JT = 2 16-row MFMA tiles per wave),
//            SW = 128; weights 32 x 576 = 144 VGPRs per wave;
//   CIN 128: 1 pixel group of 64 x 4 channel quarters of 16 (JT = 1), SW = 64; weights
//            16 x 1152 = 144 VGPRs per wave; each B fragment then feeds 1 MFMA per (tile, tap).
// Every source half of an input row is the CIN 64 row image (SW + 2 halo pixels x 128 B,
// swizzled), so the fragment addressing is shared.
template <int CIN> struct C3R {
  static constexpr int NSRC = CIN / 64;
  static constexpr int JT = 2 / NSRC;                 // 16-row output tiles per wave
  static constexpr int NG = 2 / NSRC;                 // 64-pixel groups per block
  static constexpr int SW = 64 * NG;                  // strip width
  static constexpr int OPW = 16 * JT;                 // output channels per wave
  static constexpr int NC = CIN / 32;                 // 32-channel K chunks per tap
  static constexpr int NI = (SW + 2 + 7) / 8;         // LDS-DMA instructions per source half
  static constexpr int HALF = NI * 1024;
  static constexpr int ROW = NSRC * HALF;             // one ring slot
  static constexpr int NQ = NSRC * NI;                // DMA instructions per row (over 4 waves)
  static constexpr int TERMS = C3R_SLOTS * ROW;       // folded epilogue terms: 64 x (scale, shift)
  static constexpr int SMEM = TERMS + 512;
};
}  // namespace

// DAC_CONV3R=0 turns the kernel off (A/B); dac_conv3r_enable does the same at run time
// (tools/convbench; not part of the public ABI).
static int g_conv3r_on = getenv("DAC_CONV3R") ? atoi(getenv("DAC_CONV3R")) : 1;
extern "C" void dac_conv3r_enable(int on) { g_conv3r_on = on; }

bool conv3r_ok(const ConvArgs& a) {
  if (!g_conv3r_on) return false;
  if (!(a.Cin == 64 || a.Cin == 128) || a.Cout != 64 || a.K != 9 * a.Cin) return false;
  const int SW = a.Cin == 64 ? C3R<64>::SW : C3R<128>::SW;
  // Fused 1x1 res_conv (y2 = x w2^T, module_util.py:142,153): the CIN 128 form, plain weights.
  if (a.y2 && !(a.Cin == 128 && a.w2 && !a.w2_dual && !a.bias2 && a.ldy2 % 4 == 0)) return false;
  // Source halves: channels [0, 64) and [64, 128) each whole in x1 or in x2.
  const bool one = a.x2 == nullptr || a.C1 >= a.Cin;
  if (!one && !(a.C1 == 64 && a.Cin == 128 && a.ld2 % 8 == 0)) return false;
  return !a.up && !a.uph && a.cwrap == 0 && !a.ys8 && !a.xs8 && a.amode == 0 && a.w_bstride == 0 && !a.ln_g &&
         !a.lnf_cs && !a.gna_stats && a.ksplit <= 1 && (a.act == ACT_NONE || a.act == ACT_SILU) && !a.res2 &&
         !a.bbias && !(a.res1 && a.y2) && a.Wo % SW == 0 && a.Wo >= 256 && a.Hs == a.Ho && a.Ws == a.Wo &&
         a.ld1 % 8 == 0 && a.ldy % 8 == 0 && (!a.res1 || a.ldr1 % 8 == 0) &&
         (!a.ss || (a.ss_ld % 4 == 0 && ((uintptr_t)a.ss & 15) == 0)) &&
         // per-image buffer descriptors: 31-bit byte offsets within ONE image (never the batch)
         ((size_t)a.Hs * a.Ws + 1) * a.ld1 * 2 < ((size_t)1 << 31) &&
         (one || ((size_t)a.Hs * a.Ws + 1) * a.ld2 * 2 < ((size_t)1 << 31));
}

// RES: block2's residual (res1); SILU: the activation; FUSE: the fused 1x1 res_conv output y2 —
// compile-time, so each instantiation holds only its own epilogue's registers (the kernel runs at
// the 256-VGPR limit of 2 waves per SIMD).
template <typename T, int CIN, bool RES, bool SILU, bool FUSE>
__global__ void __launch_bounds__(256, 2) conv3r_kernel(ConvArgs a, int RB) {
  kernarg_touch<sizeof(ConvArgs) + 4>();                     // every kernarg line once, one wait (common.h)
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  using G = C3R<CIN>;
  constexpr int JT = G::JT, NC = G::NC, SW = G::SW, NI = G::NI;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave / (4 / G::NG);               // pixel group
  const int ob = G::OPW * (wave % (4 / G::NG));   // first output channel of this wave
  const int lr = lane & 15, lg = lane >> 4;

  // Band of this block (XCD-contiguous: blocks b and b + 8 share an XCD, so each XCD walks a
  // contiguous range of bands, strips fastest — neighbouring bands share their halo rows in L2).
  const int nbands = gridDim.x;
  const int bid = nbands % 8 == 0 ? (blockIdx.x & 7) * (nbands >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int S = a.Wo / SW, nrb = a.Ho / RB;
  const int strip = bid % S, rb = (bid / S) % nrb, img = bid / (S * nrb);
  const int x0 = strip * SW, r0 = rb * RB;

  // Weights -> VGPRs, once: A fragment (K step ks = tap * NC + c32, tile j) of lane (lr, lg) is
  // weight row n(lr, j), 8 channels from 32 c32 + 8 lg of tap ks / NC. JT = 2: row
  // ob + 8 (lr >> 2) + 4 j + (lr & 3), so each lane's accumulators (tile i, j, element e) are
  // channels ob + 8 lg + 4 j + e of pixel 4 lr + i, 8 consecutive channels; JT = 1: row ob + lr,
  // the lane's 4 accumulators channels ob + 4 lg + e.
  auto wrow = [&](int j) { return JT == 2 ? ob + 8 * (lr >> 2) + 4 * j + (lr & 3) : ob + lr; };
  u32x4 W[9 * NC][JT];
  u32x4 WR[FUSE ? NC : 1][JT];
  {
    const T* w = reinterpret_cast<const T*>(a.w);
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int n = wrow(j);
#pragma unroll
      for (int ks = 0; ks < 9 * NC; ++ks)
        W[ks][j] = *reinterpret_cast<const u32x4*>(w + (size_t)n * (9 * CIN) + (ks / NC) * CIN + (ks % NC) * 32 + 8 * lg);
      if constexpr (FUSE) {
        const T* w2 = reinterpret_cast<const T*>(a.w2);
#pragma unroll
        for (int c = 0; c < NC; ++c) WR[c][j] = *reinterpret_cast<const u32x4*>(w2 + (size_t)n * CIN + c * 32 + 8 * lg);
      }
    }
  }
  // Wait for them HERE, with the builtin (which the compiler's wait insertion sees): otherwise it
  // places the first-use waits of W inside the row loop, where every row they would execute again
  // as counted vmcnt waits on the row's freshly issued DMA (a full DMA round trip per row).
  __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)

  // LDS-DMA of input row ir into its ring slot: instruction q (q = wave + 4 k) fills source half
  // q / NI, physical slots 8 (q % NI) .. + 7; this lane fills slot 8 (q % NI) + lane / 8,
  // physical chunk lane % 8, i.e. halo pixel phys(slot), logical chunk chunk(slot, lane % 8)
  // (recomputed per row: registers are the scarce resource here, VALU is not). Each source half
  // has one buffer descriptor per image, based one pixel before the image.
  const bool one = a.x2 == nullptr || a.C1 >= a.Cin;
  const int ldb0 = a.ld1 * 2, ldb1 = one ? ldb0 : a.ld2 * 2;
  const char* xsrc0 = reinterpret_cast<const char*>(a.x1) + (size_t)img * a.Hs * a.Ws * ldb0 - ldb0;
  const char* xsrc1 = one ? xsrc0 + 128
                          : reinterpret_cast<const char*>(a.x2) + (size_t)img * a.Hs * a.Ws * ldb1 - ldb1;
  const int xbytes0 = (a.Hs * a.Ws + 1) * ldb0, xbytes1 = (a.Hs * a.Ws + 1) * ldb1 - (one ? 128 : 0);
  const bool lpad = x0 == 0, rpad = x0 + SW == a.Wo;
  auto issue_row = [&](int ir) {
    const bool ok = (unsigned)ir < (unsigned)a.Hs;
    char* dst = smem + (ir & 3) * G::ROW;
#pragma unroll
    for (int k = 0; k < (G::NQ + 3) / 4; ++k) {
      const int q = wave + 4 * k;
      if (q < G::NQ) {
        const bool h1 = q >= NI;                   // source half (wave-uniform)
        const int qq = h1 ? q - NI : q, ldb = h1 ? ldb1 : ldb0;
        const int P = 8 * qq + (lane >> 3), p = c3r_phys(P);
        const bool pad = p >= SW + 2 || (lpad && p == 0) || (rpad && p == SW + 1);
        const int v = (ok && !pad) ? p * ldb + c3r_chunk(P, lane & 7) * 16 : (int)C3R_OOB;
        buf_lds16(h1 ? xsrc1 : xsrc0, h1 ? xbytes1 : xbytes0, dst + q * 1024, v, ok ? (ir * a.Ws + x0) * ldb : 0);
      }
    }
  };

  // B-fragment byte offsets inside a source half. Fragment s < 4 is halo pixel
  // p = 64 g + 4 lr + s, whose physical slot is p ^ (lr & 1) and chunk swizzle (16 g + lr) & 7;
  // s = 4, 5 the same with lr + 1. So offset(s, c) = base[s >> 2] ^ ((s & 3) << 7) ^ (c << 6)
  // for the half's 32-channel chunk c: two registers (VALU is cheap here, VGPRs are not), the XOR
  // terms touching only the slot's low pixel bits and bit 2 of the chunk index.
  int bbase[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = lr + u;                        // 4 q = first pixel of the quad (relative to 64 g)
    bbase[u] = (64 * g + 4 * q) * 128 + ((q & 1) << 7) + ((lg ^ ((16 * g + q) & 7)) << 4);
  }

  // Epilogue terms: (bias, 1 + scale, shift) folded once per block (the block stays inside image
  // img) into LDS, read back per row from LDS — no global loads (and no compiler-inserted vmcnt
  // waits) in the row loop, and no registers held across the MFMAs.
  constexpr int EV = 4 * JT;                     // output values per lane and tile
  const int nb = ob + EV * lg;                   // the lane's first output channel
  float* terms = reinterpret_cast<float*>(smem + G::TERMS);
  if (threadIdx.x < 64) {
    const int n = threadIdx.x;
    float sc = 1.f, sh = 0.f;
    if (a.ss) {
      sc += a.ss[(size_t)img * a.ss_ld + n];
      sh = a.ss[(size_t)img * a.ss_ld + a.Cout + n];
    }
    epi_fold(a.bias ? a.bias[n] : 0.f, sc, sh, SILU);
    terms[n] = sc;
    terms[64 + n] = sh;
  }
  T* y = reinterpret_cast<T*>(a.y);
  T* y2 = FUSE ? reinterpret_cast<T*>(a.y2) : nullptr;
  const T* r1 = RES ? reinterpret_cast<const T*>(a.res1) : nullptr;
  __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): the terms' loads (see the weights)
  // Vector-memory ops a row's epilogue issues after the next row's DMA: its output stores.
  constexpr int NST = 4 * (FUSE ? 2 : 1);

  issue_row(r0 - 1);
  issue_row(r0);
  issue_row(r0 + 1);
  for (int r = r0; r < r0 + RB; ++r) {
    // Rows r - 1 .. r + 1 landed (this wave's pieces: every vector-memory op older than the
    // previous row's NST output stores), then the barrier publishes the other waves' pieces and
    // frees the slot of row r - 2 for row r + 2.
    if (r == r0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(NST) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (r + 2 <= r0 + RB) issue_row(r + 2);
    // This row's residual rows, requested now (inline asm: invisible to the compiler's wait
    // insertion) so they land under the MFMAs; waited for by the counted wait below.
    const size_t m0 = ((size_t)img * a.Ho + r) * a.Wo + x0 + 64 * g + 4 * lr;
    u32x4 rv[RES ? 4 : 1];
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < 4; ++i) ld_asm(rv[i], r1 + (m0 + i) * a.ldr1 + nb);
    }

    f32x4 acc[4][JT];
    f32x4 accr[FUSE ? 4 : 1][JT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JT; ++j) {
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (FUSE) accr[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const char* row = smem + ((r + kh - 1) & 3) * G::ROW;
#pragma unroll
      for (int c32 = 0; c32 < NC; ++c32) {
        // (A scheduling fence per group: hoisting the next group's fragment reads above these MFMAs
        // would take 24 more VGPRs than the 256 two waves per SIMD leave; the SIMD partner wave
        // covers the LDS latency at the group start instead.)
        __builtin_amdgcn_sched_barrier(0);
        const char* hrow = row + (c32 >> 1) * G::HALF;
        const int c = c32 & 1;
        u32x4 F[6];
#pragma unroll
        for (int s = 0; s < 6; ++s) F[s] = *reinterpret_cast<const u32x4*>(hrow + (bbase[s >> 2] ^ ((s & 3) << 7) ^ (c << 6)));
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JT; ++j) Mma<T>::run(acc[i][j], W[(kh * 3 + kw) * NC + c32][j], F[i + kw]);
        if constexpr (FUSE) {
          if (kh == 1) {                           // the centre tap: the 1x1 res_conv's input
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < JT; ++j) Mma<T>::run(accr[i][j], WR[c32][j], F[i + 1]);
          }
        }
      }
    }

    // Epilogue: tile i of lane (lr, lg) is pixel x0 + 64 g + 4 lr + i, channels nb .. nb + EV - 1.
    __builtin_amdgcn_sched_barrier(0);             // (no MFMA of this row sinks past the wait)
    if constexpr (RES) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the residual rows (and row r + 2's DMA)
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(rv[i]));
    }
    float fs[EV], fh[EV];
    {
      const f32x4* tv = reinterpret_cast<const f32x4*>(terms + nb);
#pragma unroll
      for (int q = 0; q < JT; ++q) {
        const f32x4 s0 = tv[q], h0 = tv[16 + q];
#pragma unroll
        for (int e = 0; e < 4; ++e) { fs[4 * q + e] = s0[e]; fh[4 * q + e] = h0[e]; }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[EV];
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const float u = fmaf(acc[i][e >> 2][e & 3], fs[e], fh[e]);
        v[e] = SILU ? silu_log2(u) : u;
      }
      if constexpr (RES) {
#pragma unroll
        for (int w2 = 0; w2 < EV / 2; ++w2) add_pair<T>(rv[i][w2], v[2 * w2], v[2 * w2 + 1]);
      }
      if constexpr (EV == 8) {
        store_vec<T>(y + (m0 + i) * a.ldy + nb, v);
      } else {
        store4<T>(y + (m0 + i) * a.ldy + nb, v);
      }
      if constexpr (FUSE) {
        float v2[EV];
#pragma unroll
        for (int e = 0; e < EV; ++e) v2[e] = accr[i][e >> 2][e & 3];
        if constexpr (EV == 8) store_vec<T>(y2 + (m0 + i) * a.ldy2 + nb, v2);
        else store4<T>(y2 + (m0 + i) * a.ldy2 + nb, v2);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Band height: the largest divisor of Ho giving >= 512 bands (two blocks per CU on 256 CUs),
// else 1. Speed only: the result does not depend on it.
static int conv3r_rb(const ConvArgs& a, int SW) {
  const long rows = (long)a.B * a.Ho * (a.Wo / SW);
  int rb = (int)(rows / 512);
  if (rb < 1) rb = 1;
  if (rb > a.Ho) rb = a.Ho;
  while (a.Ho % rb) --rb;
  return rb;
}

template <typename T, int CIN>
static void conv3r_launch(const ConvArgs& a, hipStream_t st) {
  constexpr int SW = C3R<CIN>::SW;
  const int rb = conv3r_rb(a, SW);
  const int nb = a.B * (a.Ho / rb) * (a.Wo / SW);
  const bool silu = a.act == ACT_SILU;
  if constexpr (CIN == 128) {
    if (a.y2 && silu) conv3r_kernel<T, CIN, false, true, true><<<nb, 256, 0, st>>>(a, rb);
    else if (a.y2) conv3r_kernel<T, CIN, false, false, true><<<nb, 256, 0, st>>>(a, rb);
    else if (a.res1 && silu) conv3r_kernel<T, CIN, true, true, false><<<nb, 256, 0, st>>>(a, rb);
    else if (a.res1) conv3r_kernel<T, CIN, true, false, false><<<nb, 256, 0, st>>>(a, rb);
    else if (silu) conv3r_kernel<T, CIN, false, true, false><<<nb, 256, 0, st>>>(a, rb);
    else conv3r_kernel<T, CIN, false, false, false><<<nb, 256, 0, st>>>(a, rb);
  } else {
    if (a.res1 && silu) conv3r_kernel<T, CIN, true, true, false><<<nb, 256, 0, st>>>(a, rb);
    else if (a.res1) conv3r_kernel<T, CIN, true, false, false><<<nb, 256, 0, st>>>(a, rb);
    else if (silu) conv3r_kernel<T, CIN, false, true, false><<<nb, 256, 0, st>>>(a, rb);
    else conv3r_kernel<T, CIN, false, false, false><<<nb, 256, 0, st>>>(a, rb);
  }
}

template <typename T>
void conv3r(const ConvArgs& a, hipStream_t st) {
  if (!conv3r_ok(a)) throw std::invalid_argument("conv3r: arguments rejected by conv3r_ok");
  if (a.Cin == 64) conv3r_launch<T, 64>(a, st);
  else conv3r_launch<T, 128>(a, st);
}
template void conv3r<bf16>(const ConvArgs&, hipStream_t);
template void conv3r<f16>(const ConvArgs&, hipStream_t);

}  // namespace dac
