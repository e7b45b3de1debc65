// conv8.hip — fp8 (OCP e4m3) implicit-GEMM convolution / linear layer on the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the 16-bit MFMA rate per clock), the MX weight path of
// the fp8 handles (BASELINE configs[4]). Activations stay 16-bit (fp16, or bf16) in HBM: every A tile is
// quantized on the fly while it is staged, with one E8M0 scale per (pixel, 64-channel block),
// and the weights are quantized once at load with one E8M0 scale per (output channel,
// 64-k block). Accumulation is fp32; the epilogue is the 16-bit kernels' (conv_epi.h).
//
// Operand layout of the 16x16x128 scaled MFMA (measured on gfx950, tools/probes): lane
// (r = l & 15, g = l >> 4) supplies 32 bytes of row r; the hardware treats them as k slots
// 16g..16g+15 and 64+16g..64+16g+15, and takes the scale of the 32-slot block b of row r from
// lane r + 16b. Here lane group g carries channels 32g..32g+31 of the 128-k step (the same
// for A and B, so the slot permutation cancels), hardware blocks {0, 2} then hold channels
// 0..63 and {1, 3} channels 64..127: lane (r, g) supplies the scale of channel block g & 1.
//
// Tile: 128 pixels x 128 output channels, 4 waves of 64 x 64 (4 x 4 MFMA tiles), K steps of
// 128 (one (tap, channel range) per 64-k half: Cin % 64 == 0), two LDS buffers, register
// prefetch of the next step while the MFMAs of this one run.
#include "conv_impl.h"

namespace dac {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef short short2_t __attribute__((ext_vector_type(2)));

// e4m3 pair conversion with an E8M0 scale, per 16-bit activation type.
template <typename T> DEV short2_t cvt8(short2_t old, typename Vec8<T>::t2 v, float sc, bool hi);
template <> DEV short2_t cvt8<bf16>(short2_t old, bf16x2_t v, float sc, bool hi) {
  return hi ? __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, sc, true)
            : __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, sc, false);
}
template <> DEV short2_t cvt8<f16>(short2_t old, f16x2_t v, float sc, bool hi) {
  return hi ? __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(old, v, sc, true)
            : __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(old, v, sc, false);
}
// |x| of the largest of a lane's packed 16-bit values (sign bits cleared, compared as integers:
// both formats order non-negative values like their bit patterns) as a float.
template <typename T> DEV float abs16_to_f(uint32_t m);
template <> DEV float abs16_to_f<bf16>(uint32_t m) { return __builtin_bit_cast(float, m << 16); }
template <> DEV float abs16_to_f<f16>(uint32_t m) { return (float)__builtin_bit_cast(f16, (uint16_t)m); }

template <typename T, int KH, int KW, int S, int P>
__global__ void __launch_bounds__(256) conv8_kernel(ConvArgs a, const uint8_t* __restrict__ w8,
                                                    const uint8_t* __restrict__ ws8, int Kp) {
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  constexpr int BM = 128, BN = 128, WGM = 2, WGN = 2, TM = 4, TN = 4;
  constexpr int ROWB = 128;                                  // bytes per staged row (128 k fp8)
  constexpr int TILE = BM * ROWB;                            // 16 KB
  constexpr int PIPE = 2 * (2 * TILE + 2 * BM * 2);
  constexpr int EPR = epi_rows<BM, BN, 64>(PIPE);
  constexpr int SMEM = PIPE > EpiLds<EPR, BN>::BYTES ? PIPE : EpiLds<EPR, BN>::BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  auto sA = [&](int buf) { return smem + buf * (2 * TILE + 4 * BM); };
  auto sB = [&](int buf) { return sA(buf) + TILE; };
  auto sAs = [&](int buf) { return reinterpret_cast<uint8_t*>(sA(buf) + 2 * TILE); };
  auto sBs = [&](int buf) { return sAs(buf) + 2 * BM; };
  // 16-byte slot s of row r lives at slot s ^ ((r >> 1) & 7): the 16 rows of a fragment read
  // land on 16 distinct bank quads.
  auto swz = [](int row, int s) { return row * ROWB + ((s ^ ((row >> 1) & 7)) << 4); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int lr = lane & 15, lg = lane >> 4;
  const int HWo = a.Ho * a.Wo;
  const TileId tl = xcd_tile();
  const int M = a.B * HWo;
  const int m0 = tl.bx * BM, n0 = tl.by * BN;
  const int Hin = a.up ? 2 * a.Hs : a.Hs, Win = a.up ? 2 * a.Ws : a.Ws;
  const int nk = Kp / 128;

  // Staging role: row sr of the tile, 64-k half sh.
  const int sr = tid >> 1, sh = tid & 1;
  int pix0 = 0, ih0 = -100000, iw0 = -100000;
  {
    const int m = m0 + sr;
    if (m < M) {
      const int b = m / HWo, r = m - b * HWo;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      pix0 = b * a.Hs * a.Ws;
      ih0 = oh * S - P;
      iw0 = ow * S - P;
    }
  }
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  const int nrow = n0 + sr;
  const uint8_t* wrow = nrow < a.Cout ? w8 + (size_t)nrow * Kp : nullptr;
  const uint8_t* wsrow = nrow < a.Cout ? ws8 + (size_t)nrow * (Kp / 64) : nullptr;

  u32x4 ra[8], rb[4];
  uint32_t rbs = 127;
  auto gload = [&](int kt) {
    const int k = kt * 128 + sh * 64;
    bool ok = k < a.K;
    int tap = 0, ci = k;
    if constexpr (KH * KW > 1) { tap = k / a.Cin; ci = k - tap * a.Cin; }
    const int kh = tap / KW, kw = tap - (tap / KW) * KW;
    const int ih = ih0 + kh, iw = iw0 + kw;
    ok = ok && (unsigned)ih < (unsigned)Hin && (unsigned)iw < (unsigned)Win;
    const T* src = nullptr;
    if (ok) {
      const int shh = a.up ? (ih >> 1) : ih, sww = a.up ? (iw >> 1) : iw;
      const size_t pix = (size_t)(pix0 + shh * a.Ws + sww);
      src = ci < a.C1 ? x1 + pix * a.ld1 + ci : x2 + pix * a.ld2 + (ci - a.C1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) ra[i] = ok ? reinterpret_cast<const u32x4*>(src)[i] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      rb[i] = wrow ? reinterpret_cast<const u32x4*>(wrow + kt * 128 + sh * 64)[i] : u32x4{0u, 0u, 0u, 0u};
    rbs = wsrow ? wsrow[kt * 2 + sh] : 127u;
  };
  // Quantize the 64 staged activations (E8M0 exponent e: |x| / 2^e <= 448) and store.
  auto sstore = [&](int buf) {
    uint32_t mx = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t v = ra[i][q] & 0x7fff7fffu;
        mx = max(mx, max(v & 0xffffu, v >> 16));
      }
    const float p = abs16_to_f<T>(mx);
    int e = 0;
    if (p > 0.f) e = (int)ceilf(__log2f(p * (1.f / 448.f)));
    e = e < -126 ? -126 : (e > 126 ? 126 : e);
    const float sc = __builtin_bit_cast(float, (uint32_t)(e + 127) << 23);    // 2^e
    u32x4 q8[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // 8 16-bit values -> 8 fp8 (two dwords). The pairs are taken by shufflevector from the
      // whole 8-vector: hipcc (ROCm 7.2) miscompiles __builtin_bit_cast(bf16x2_t, ra[i][q]) fed
      // to this builtin (every call reads element 0 and the second result is dropped).
      const typename Vec8<T>::t w = __builtin_bit_cast(typename Vec8<T>::t, ra[i]);
      short2_t lo = {0, 0}, hi = {0, 0};
      lo = cvt8<T>(lo, __builtin_shufflevector(w, w, 0, 1), sc, false);
      lo = cvt8<T>(lo, __builtin_shufflevector(w, w, 2, 3), sc, true);
      hi = cvt8<T>(hi, __builtin_shufflevector(w, w, 4, 5), sc, false);
      hi = cvt8<T>(hi, __builtin_shufflevector(w, w, 6, 7), sc, true);
      q8[i >> 1][(i & 1) * 2] = __builtin_bit_cast(uint32_t, lo);
      q8[i >> 1][(i & 1) * 2 + 1] = __builtin_bit_cast(uint32_t, hi);
    }
    char* A = sA(buf);
    char* Bt = sB(buf);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      *reinterpret_cast<u32x4*>(A + swz(sr, sh * 4 + s)) = q8[s];
      *reinterpret_cast<u32x4*>(Bt + swz(sr, sh * 4 + s)) = rb[s];
    }
    sAs(buf)[sr * 2 + sh] = (uint8_t)(e + 127);
    sBs(buf)[sr * 2 + sh] = (uint8_t)rbs;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* A = sA(cur);
    const char* Bt = sB(cur);
    i32x8 fa[TM], fb[TN];
    int sa[TM], sb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * 64 + i * 16 + lr;
      const u32x4 p0 = *reinterpret_cast<const u32x4*>(A + swz(row, 2 * lg));
      const u32x4 p1 = *reinterpret_cast<const u32x4*>(A + swz(row, 2 * lg + 1));
      fa[i] = i32x8{(int)p0[0], (int)p0[1], (int)p0[2], (int)p0[3], (int)p1[0], (int)p1[1], (int)p1[2], (int)p1[3]};
      sa[i] = sAs(cur)[row * 2 + (lg & 1)];
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * 64 + j * 16 + lr;
      const u32x4 p0 = *reinterpret_cast<const u32x4*>(Bt + swz(row, 2 * lg));
      const u32x4 p1 = *reinterpret_cast<const u32x4*>(Bt + swz(row, 2 * lg + 1));
      fb[j] = i32x8{(int)p0[0], (int)p0[1], (int)p0[2], (int)p0[3], (int)p1[0], (int)p1[1], (int)p1[2], (int)p1[3]};
      sb[j] = sBs(cur)[row * 2 + (lg & 1)];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i][j], 0, 0, 0, sa[i], 0, sb[j]);
    if (kt + 1 < nk) {
      // Buffer cur^1 was last read in step kt - 1, before that step's closing barrier.
      sstore(cur ^ 1);
      __syncthreads();
    }
  }
  __syncthreads();                   // the epilogue's LDS tile overlays the last step's buffer
  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;
  const int bimg = (m0 / HWo == mlast / HWo) ? m0 / HWo : -1;
  conv_epilogue_lds<T, BM, BN, WGM, WGN, EPR>(a, acc, smem, M, LinearRows{m0}, n0, HWo, bimg);
}

bool conv8_ok(const ConvArgs& a, int kh, int kw, int s, int p) {
  const bool shape = (kh == 3 && kw == 3 && s == 1 && p == 1) || (kh == 1 && kw == 1 && s == 1 && p == 0) ||
                     (kh == 4 && kw == 4 && s == 2 && p == 1);
  return shape && a.zero && a.Cin % 64 == 0 && (a.x2 == nullptr || a.C1 % 64 == 0) && a.amode == 0 &&
         a.w_bstride == 0 && !a.ln_g && !a.lnf_cs && !a.gna_stats && a.cwrap == 0 && a.Cout >= 32 && (kh > 1 || a.up == 0);
}

template <typename T>
void conv8(const ConvArgs& a, int kh, int kw, int s, int p, const uint8_t* w8, const uint8_t* ws8, int Kp,
           hipStream_t st) {
  const int M = a.B * a.Ho * a.Wo;
  dim3 g((M + 127) / 128, (a.Cout + 127) / 128, 1);
  if (kh == 3) conv8_kernel<T, 3, 3, 1, 1><<<g, 256, 0, st>>>(a, w8, ws8, Kp);
  else if (kh == 1) conv8_kernel<T, 1, 1, 1, 0><<<g, 256, 0, st>>>(a, w8, ws8, Kp);
  else conv8_kernel<T, 4, 4, 2, 1><<<g, 256, 0, st>>>(a, w8, ws8, Kp);
}
template void conv8<bf16>(const ConvArgs&, int, int, int, int, const uint8_t*, const uint8_t*, int, hipStream_t);
template void conv8<f16>(const ConvArgs&, int, int, int, int, const uint8_t*, const uint8_t*, int, hipStream_t);

}  // namespace dac
