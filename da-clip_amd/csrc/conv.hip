// conv.hip — MFMA implicit-GEMM convolution for gfx950 (NHWC activations).
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
#include "common.h"
#include "kernels.h"

namespace dac {

template <typename T, int BM, int BN, int WGM, int WGN, int KH, int KW, int S, int P>
__global__ void __launch_bounds__(256) conv_kernel(ConvArgs a) {
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int BKE = 128 / sizeof(T);
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int AV = BM / 32;
  constexpr int BV = (BN + 31) / 32;
  constexpr int KSTEPS = BKE / Mma<T>::KSTEP;
  static_assert(WGM * WGN == 4 && TM >= 1 && TN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * 128];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int HWo = a.Ho * a.Wo;
  // Batched grid (per-image weights): rows of image blockIdx.z only.
  const bool batched = a.w_bstride > 0;
  const int M = batched ? (blockIdx.z + 1) * HWo : a.B * HWo;
  const int m0 = (batched ? blockIdx.z * HWo : 0) + blockIdx.x * BM, n0 = blockIdx.y * BN;
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
  const T* wgt = reinterpret_cast<const T*>(a.w) + (batched ? blockIdx.z * a.w_bstride : 0);

  u32x4 ra[AV], rb[BV];
  const int nk = (a.K + BKE - 1) / BKE;

  auto gload = [&](int kt) {
    const int k = kt * BKE + slot * VE;
    const bool kv = k < a.K;
    int kpos = k / a.Cin;
    const int ci = k - kpos * a.Cin;
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

  // Epilogue.
  T* y = reinterpret_cast<T*>(a.y);
  const T* r1 = reinterpret_cast<const T*>(a.res1);
  const T* r2 = reinterpret_cast<const T*>(a.res2);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + lg * 4 + r;
      if (m >= M) continue;
      const int b = m / HWo;
      if (a.act == ACT_GEGLU) {
        if constexpr (TN % 2 == 0) {
#pragma unroll
          for (int j = 0; j < TN; j += 2) {
            const int nx = n0 + wn * WTN + j * 16 + lr;     // "x" half of the pair
            const int no = (n0 + wn * WTN + j * 16) / 2 + lr; // output column
            if (nx >= a.Cout) continue;
            float vx = acc[i][j][r], vg = acc[i][j + 1][r];
            if (a.bias) { vx += a.bias[nx]; vg += a.bias[nx + 16]; }
            float v = vx * gelu_f(vg);
            if (r1) v += to_f(r1[(size_t)m * a.ldr1 + no]);
            y[(size_t)m * a.ldy + no] = from_f<T>(v);
          }
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + lr;
        if (n >= a.Cout) continue;
        float v = acc[i][j][r];
        if (a.bias) v += a.bias[n];
        if (a.ss) {
          const float* s = a.ss + (size_t)b * a.ss_ld;
          v = v * (s[n] + 1.f) + s[a.Cout + n];
        }
        if (a.act == ACT_SILU) v = silu_f(v);
        else if (a.act == ACT_GELU) v = gelu_f(v);
        if (r1) v += to_f(r1[(size_t)m * a.ldr1 + n]);
        if (r2) v += to_f(r2[(size_t)m * a.ldr2 + n]);
        if (a.bbias) v += a.bbias[(size_t)b * a.bb_ld + n];
        y[(size_t)m * a.ldy + n] = from_f<T>(v);
      }
    }
  }
}

template <typename T, int KH, int KW, int S, int P>
static void conv_dispatch(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.Ho * a.Wo;
  const bool batched = a.w_bstride > 0;
  const int Mg = batched ? a.Ho * a.Wo : M;
  const int gz = batched ? a.B : 1;
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

template <typename T>
void conv(const ConvArgs& a, int kh, int kw, int s, int p, hipStream_t st) {
  if (kh == 3 && kw == 3 && s == 1 && p == 1) conv_dispatch<T, 3, 3, 1, 1>(a, st);
  else if (kh == 1 && kw == 1 && s == 1 && p == 0) conv_dispatch<T, 1, 1, 1, 0>(a, st);
  else if (kh == 4 && kw == 4 && s == 2 && p == 1) conv_dispatch<T, 4, 4, 2, 1>(a, st);
  else if (kh == 7 && kw == 7 && s == 1 && p == 3) conv_dispatch<T, 7, 7, 1, 3>(a, st);
  else if (kh == 32 && kw == 32 && s == 32 && p == 0) conv_dispatch<T, 32, 32, 32, 0>(a, st);
  else if (kh == 14 && kw == 14 && s == 14 && p == 0) conv_dispatch<T, 14, 14, 14, 0>(a, st);
  else __builtin_trap();
}

template void conv<float>(const ConvArgs&, int, int, int, int, hipStream_t);
template void conv<bf16>(const ConvArgs&, int, int, int, int, hipStream_t);

}  // namespace dac
