// conv_down.hip — the UNet's Downsample convs for 16-bit (bf16 / f16) handles: 4x4, stride 2, pad 1
// (module_util.py:107-108 `nn.Conv2d(dim, dim_out, 4, 2, 1)`), Cin % 32 == 0, Cout % 64 == 0.
//
// The generic implicit GEMM gathered one input pixel per (output pixel, tap): 16 taps x 128 B
// per output pixel through LDS-DMA, 4x the input for a stride-2 4x4 kernel (51 us at 256^2).
// Here a block owns 128 output pixels (one row segment, or 128 / Wo whole rows) x 64 output
// channels, and each stage (32-channel chunk, kernel row kh) DMAs the needed input row band
// ONCE — 2 * width + 2 pixels per output row — with the pixels deinterleaved into an even and
// an odd half: output pixel x, tap kw reads input pixel 2x + kw - 1, i.e. consecutive LDS rows
// of one half for every kw (the stride-2 reads of an interleaved row can only reach 8 of the
// 16 bank quads). The 4 kw taps' weights (4 x 64 rows) come with the stage.
// MFMA operands swapped (weights as A, rows permuted by wperm64) so each lane ends with 16
// consecutive channels of one pixel: the register epilogue epi_regs16 (bias, scale/shift, SiLU,
// residuals) writes 16-byte rows. 4 waves x 32 pixels (2 pixel tiles) x 64 channels, 2-stage
// LDS ring, one barrier per stage.
#include "common.h"
#include "kernels.h"
#include "conv_impl.h"

namespace dac {

constexpr int CD_PIX = 128;                        // output pixels per tile
constexpr int CD_AROWS = 272;                      // >= 128/Wo rows x (2 Wo + 2) halo pixels
constexpr int CD_BROWS = 256;                      // 4 taps x 64 output channels
constexpr int CD_STAGE = (CD_AROWS + CD_BROWS) * 64;
constexpr int CD_NA = CD_AROWS / 16, CD_NB = CD_BROWS / 16;   // DMA instructions per stage

bool conv_down_ok(const ConvArgs& a) {
  const bool wo_ok = a.Wo >= 32 && (a.Wo % CD_PIX == 0 || (CD_PIX % a.Wo == 0 && (a.Wo & (a.Wo - 1)) == 0));
  const bool epi = (a.act == ACT_NONE || a.act == ACT_SILU) && a.ldy % 8 == 0 && (!a.res1 || a.ldr1 % 8 == 0) &&
                   (!a.res2 || a.ldr2 % 8 == 0) && (!a.ss || (a.ss_ld % 4 == 0 && ((uintptr_t)a.ss & 15) == 0));
  return a.zero && !a.up && a.amode == 0 && a.w_bstride == 0 && a.cwrap == 0 && !a.ln_g && !a.y2 &&
         a.Cin % 32 == 0 && a.Cout % 64 == 0 && a.K == 16 * a.Cin && a.C1 >= a.Cin && !a.x2 &&
         a.ld1 % 8 == 0 && a.Ho * 2 == a.Hs && a.Wo * 2 == a.Ws && wo_ok &&
         (a.Ho * a.Wo) % CD_PIX == 0 && epi;
}

template <typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_down_kernel(ConvArgs a) {
  kernarg_touch<sizeof(ConvArgs)>();                     // every kernarg line once, one wait (common.h)
  StampGuard stamp_guard(a.stamp);                          // in-graph timing (null: off)
  __shared__ __attribute__((aligned(1024))) char smem[2 * CD_STAGE];
  using SB = RowSwz<4, 1>;                         // 64-byte rows read 16 consecutive at a time
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const TileId tl = xcd_tile();                    // by = output-channel tile (fastest)
  const int n0 = tl.by * 64;
  const long m0 = (long)tl.bx * CD_PIX;            // first output pixel of the tile
  const int HWo = a.Ho * a.Wo;
  const int b = (int)(m0 / HWo);
  const int r0 = (int)(m0 - (long)b * HWo);
  const int oh0 = r0 / a.Wo, ow0 = r0 - oh0 * a.Wo;
  const int segw = a.Wo < CD_PIX ? a.Wo : CD_PIX;  // output pixels per tile row
  const int nrow = CD_PIX / segw;                  // output rows per tile
  const int hrow = 2 * segw + 2;                   // halo pixels per output row
  const int half = segw + 1;                       // even / odd half of a halo row
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const char* xs = reinterpret_cast<const char*>(a.x1);
  const size_t ldb = (size_t)a.ld1 * 2;

  // A DMA: LDS row R of output row q = R / hrow, position u = R % hrow: u < half is even halo
  // pixel 2u, else odd halo pixel 2(u - half) + 1; halo pixel p is input column 2*ow0 - 1 + p.
  int a_q[(CD_NA + 3) / 4], a_iw[(CD_NA + 3) / 4], a_sl[(CD_NA + 3) / 4];
#pragma unroll
  for (int k = 0; k < (CD_NA + 3) / 4; ++k) {
    const int R = (wave + 4 * k) * 16 + (lane >> 2);
    const int q = R / hrow, u = R - q * hrow;
    const int p = u < half ? 2 * u : 2 * (u - half) + 1;
    a_q[k] = (q < nrow && wave + 4 * k < CD_NA) ? q : -1;
    a_iw[k] = 2 * ow0 - 1 + p;
    a_sl[k] = SB::slot(R, lane & 3) * 16;
  }
  // B DMA: row = kw * 64 + rho (rho = MFMA row, output channel n0 + wperm64(rho)).
  const T* b_src[CD_NB / 4];
  int b_sl[CD_NB / 4];
#pragma unroll
  for (int k = 0; k < CD_NB / 4; ++k) {
    const int row = (wave + 4 * k) * 16 + (lane >> 2);
    const int kw = row >> 6, n = n0 + wperm64(row & 63);
    b_src[k] = reinterpret_cast<const T*>(a.w) + (size_t)n * a.K + kw * a.Cin;
    b_sl[k] = SB::slot(row, lane & 3) * 8;
  }
  auto issue = [&](int c, int kh, int buf) {
    char* st = smem + buf * CD_STAGE;
    const int ci0 = c * 32;
#pragma unroll
    for (int k = 0; k < (CD_NA + 3) / 4; ++k) {
      if (wave + 4 * k < CD_NA) {                  // wave-uniform
        const char* src = zero;
        if (a_q[k] >= 0) {
          const int ih = 2 * (oh0 + a_q[k]) - 1 + kh, iw = a_iw[k];
          if ((unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws)
            src = xs + ((size_t)(b * a.Hs + ih) * a.Ws + iw) * ldb + ci0 * 2 + a_sl[k];
        }
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(st + (wave + 4 * k) * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < CD_NB / 4; ++k) {
      const char* src = reinterpret_cast<const char*>(b_src[k] + kh * 4 * a.Cin + ci0 + b_sl[k]);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(st + CD_AROWS * 64 + (wave + 4 * k) * 1024), 16, 0, 0);
    }
  };

  // This wave's output pixels t = 32 * wave + 16 i + lr: output row q, column x.
  int arow[2][4];                                  // [pixel tile][kw] LDS row of the A fragment
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int t = 32 * wave + 16 * i + lr;
    const int q = t / segw, x = t - q * segw;
#pragma unroll
    for (int kw = 0; kw < 4; ++kw) arow[i][kw] = q * hrow + ((kw & 1) ? half : 0) + x + (kw >> 1);
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunk = a.Cin / 32, S = 4 * nchunk;
  issue(0, 0, 0);
  for (int s = 0; s < S; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 1 < S) issue((s + 1) >> 2, (s + 1) & 3, buf ^ 1);
    const char* st = smem + buf * CD_STAGE;
#pragma unroll
    for (int kw = 0; kw < 4; ++kw) {
      u32x4 fa[2], fw[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int R = arow[i][kw];
        fa[i] = *reinterpret_cast<const u32x4*>(st + R * 64 + (SB::slot(R, lg) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = kw * 64 + 16 * j + lr;
        fw[j] = *reinterpret_cast<const u32x4*>(st + CD_AROWS * 64 + row * 64 + (SB::slot(row, lg) << 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], fw[j], fa[i]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nb = n0 + 16 * lg;
  float bi[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) bi[e] = a.bias ? a.bias[nb + e] : 0.f;
  // Pixel tile i, lane lr: output pixel m0 + 32 * wave + 16 i + lr (tiles never straddle images).
  epi_regs16<T, 2>(a, acc, bi, nb, b, [&](int i) { return (size_t)(m0 + 32 * wave + 16 * i + lr); });
}

template <typename T>
void conv_down(const ConvArgs& a, hipStream_t st) {
  const int npix = (int)((long)a.B * a.Ho * a.Wo / CD_PIX);
  conv_down_kernel<T><<<dim3(npix, a.Cout / 64, 1), 256, 0, st>>>(a);
}

template void conv_down<bf16>(const ConvArgs&, hipStream_t);
template void conv_down<f16>(const ConvArgs&, hipStream_t);

}  // namespace dac
