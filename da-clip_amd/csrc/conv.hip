// conv.hip — tap-shape switch of the implicit-GEMM conv; kernels live in conv_impl.h and are
// instantiated in conv_k3.hip / conv_k1.hip / conv_kx.hip.
#include "common.h"
#include "kernels.h"
#include "conv_epi.h"

namespace dac {

int g_conv3_force = -1;
int g_conv2_force = 0;
// DAC_CONV2_FORCE32=k: 1x1 configuration k for the small-image plain GEMMs (256 <= Ho*Wo <= 1024:
// the SpatialTransformer level; GEGLU projections and the LN / GroupNorm folds keep their tiles).
// Default 18, swapped 128x128 tiles with a 4-stage ring: with the lowest levels split into two
// half-batch branches it measured +0.6-0.8 % over the 64x128 tiles (four interleaved pairs,
// DESIGN.md §9); 0 = the general dispatch.
int g_conv2_force32 = getenv("DAC_CONV2_FORCE32") ? atoi(getenv("DAC_CONV2_FORCE32")) : 18;
int g_conv3_buf = getenv("DAC_CONV3_BUF") ? atoi(getenv("DAC_CONV3_BUF")) : 1;
int g_conv3h_on = getenv("DAC_CONV3H") ? atoi(getenv("DAC_CONV3H")) : 0;
int g_c3i_st = getenv("DAC_C3I_ST") ? atoi(getenv("DAC_C3I_ST")) : 3;
extern "C" void dac_c3i_st(int v) { g_c3i_st = v; }
// GEGLU projections on swapped tiles with the register epilogue: 0 off (the 256x256 LDS-epilogue
// tile), 1 256x256 (16 waves), 2 128x256, 3 256x128, 4 128x128 (DAC_GEGLU_SW; convbench forces
// 20..23 = configurations 1..4).
int g_geglu_sw = getenv("DAC_GEGLU_SW") ? atoi(getenv("DAC_GEGLU_SW")) : 1;
extern "C" void dac_conv3_force(int v) { g_conv3_force = v; }
extern "C" void dac_conv2_force(int v) { g_conv2_force = v; }

template <typename T, int KH, int KW, int S, int P>
void conv_dispatch(const ConvArgs& a, hipStream_t st);

// Kernel variant conv_dispatch selects (mirrors its logic); used to label timed launches:
// 0/1/2 = v1 256x16 / 256x64 / 128x128, 3/4/5 = v2 256x64 / 256x128 / 128x128,
// 6/7 = v3 (row-halo 3x3, 64-byte rows, 4 waves) 128x64 / 128x128, 10/11 = v3 (128-byte rows,
// 8 waves) 256x64 / 128x128, 8 = v2 single-stage 1x1 (K = one tile) 128x64, 12 = v4 (3x3
// interleaved-row tiles) 256x64, 13 = v2 7x7 row-tap layout (bf16, Cin = 8), 14 = v4 256x16
// (narrow Cout), 15 / 16 / 17 / 18 = v2 1x1 128x256 (GEGLU) / 256x256 / 64x128 / 128x64,
// 2-stage, 20 = v4 with 32-pixel wave tiles 128x64, 21 = v5 weight-stationary 3x3 (64 -> 64),
// 22 / 23 = conv_edge.hip init_conv (7x7, Cin 8, Cout 64) / final_conv (3x3, Cout <= 4),
// 24 = conv_down.hip (4x4 stride-2 Downsample), 25 = v6 2-D halo 3x3 (conv3h_kernel), 26 = v4
// row-phase upsample conv (ConvArgs::uph; labelled by the engine, not returned here), 27 = conv3r
// register-stationary 3x3 (64 -> 64, conv3r.hip).
int conv3_rw_host(const ConvArgs& a, int BM) {
  const int Wo = a.Wo, Ho = a.Ho;
  if (Wo <= 0 || (Wo & (Wo - 1))) return Wo % BM == 0 ? BM : 0;
  const int RW = Wo < BM ? Wo : BM;
  if (RW < 16 || Ho % (BM / RW)) return 0;
  return RW;
}
int conv_variant(const ConvArgs& a, int kh, int elem_bytes) {
  const int BKE = 128 / elem_bytes;
  const bool V2 = kh == 1 || kh == 3 || kh == 4;
  const bool batched = a.w_bstride > 0;
  const int Mg = batched ? a.Ho * a.Wo : a.B * a.Ho * a.Wo;
  const int gz = batched ? a.B : 1;
  const bool v2ok = V2 && a.zero && a.Cin % BKE == 0 && a.amode == 0 && a.Cout > 16;
  const int VEh = 16 / elem_bytes;
  const bool epi_min = (a.act == ACT_NONE || a.act == ACT_SILU) && a.Cout % VEh == 0 && a.ldy % VEh == 0 &&
                       (!a.res1 || a.ldr1 % VEh == 0) && (!a.res2 || a.ldr2 % VEh == 0);
  if (kh == 7 && elem_bytes == 2 && conv7_ok(a)) return 22;
  if (kh == 3 && elem_bytes == 2 && g_conv3_force < 0 && conv3n_ok(a)) return 23;
  if (kh == 4 && elem_bytes == 2 && g_conv3_force < 0 && conv_down_ok(a)) return 24;
  if (kh == 7 && elem_bytes == 2 && a.Cin == 8 && a.K == 7 * 8 * 8 && a.zero && a.amode == 0 && !batched &&
      !a.x2)
    return 13;
  if (kh == 3 && a.Cout <= 16 && a.zero && a.amode == 0 && !batched && g_conv3_force < 0 &&
      (a.act == ACT_NONE || a.act == ACT_SILU) && a.Cin % (64 / elem_bytes) == 0 && conv3_rw_host(a, 256) > 0 &&
      conv3_rw_host(a, 256) % 64 == 0)
    return 14;
  if (kh == 3 && (g_conv3_force == 60 || g_conv3_force == 61 || (g_conv3_force < 0 && g_conv3h_on == 2) ||
                  (g_conv3_force < 0 && g_conv3h_on == 1 && a.Cin >= 128 && !a.res1 && !a.res2 && !a.bbias)) &&
      conv3h_ok(a, elem_bytes))
    return 25;
  if (kh == 3 && elem_bytes == 2 && (g_conv3_force < 0 || g_conv3_force == 70) && conv3r_ok(a)) return 27;
  if (kh == 3 && elem_bytes == 2 && (g_conv3_force < 0 || (g_conv3_force >= 30 && g_conv3_force < 40)) && conv3w_ok(a)) return 21;
  if (kh == 3 && v2ok && !batched && epi_min && conv3_rw_host(a, 256) > 0 && g_conv3_force < 0) {
    const int RW = conv3_rw_host(a, 256);
    const bool kok = (a.C1 >= a.Cin || a.C1 % (64 / elem_bytes) == 0) && a.Cin % (64 / elem_bytes) == 0;
    if (RW % 64 == 0 && kok) return 12;
    if (kok && a.Cout <= 256 && conv3_rw_host(a, 128) > 0 && conv3_rw_host(a, 128) % 32 == 0) return 20;
  }
  if (kh == 3 && v2ok && !batched && epi_min && conv3_rw_host(a, 256) > 0) {
    if (a.Cout <= 64) return conv3_rw_host(a, 128) > 0 ? 6 : 10;
    if (conv3_rw_host(a, 128) > 0)
      return (long)(a.Ho * a.Wo / 128) * ((a.Cout + 127) / 128) >= 64 ? 7 : 11;   // per image (batch-invariant)
  }
  if (v2ok) {
    if (kh == 1 && a.K <= BKE) return 8;
    if (kh == 1 && a.Cout <= 64) return 18;
    if (a.Cout <= 64) return 3;
    if (kh == 1) {
      if (a.act == ACT_GEGLU) return 15;
      const bool minimal = a.Cout % VEh == 0 && a.ldy % VEh == 0 && (!a.res1 || a.ldr1 % VEh == 0) &&
                           (!a.res2 || a.ldr2 % VEh == 0) && (a.act == ACT_NONE || a.act == ACT_SILU) &&
                           (batched || (a.Ho * a.Wo) % 256 == 0);
      if (a.Cout >= 1024 && minimal) return 16;
      return 17;
    }
    if ((long)((Mg + 255) / 256) * ((a.Cout + 127) / 128) * gz >= 256) return 4;
    return 5;
  }
  if (a.Cout <= 16 && a.act != ACT_GEGLU) return 0;
  return a.Cout <= 64 ? 1 : 2;
}

// The fused res_conv rides on the bf16 v4 swapped-operand kernels: 256x64 tiles (variant 12)
// or, for 32-pixel rows (the 32x32 level, any Cout), 128x64 tiles.
// It mirrors every condition of the two fused conv3i_try calls in conv_dispatch (kernel choice,
// no forced configuration, the swapped tiles' 16-byte scale / shift / bias DMA); the dispatcher
// aborts if neither launches, so y2 is never left unwritten.
// Mirrors the EPI_LNF branch of conv_dispatch (conv_impl.h): 1x1, 16-bit, whole 16-byte rows,
// tiles inside one image, 64x128 swapped tiles; no GEGLU (the tile that folded it is gone).
bool conv_lnf_ok(const ConvArgs& a, int elem_bytes) {
  if (elem_bytes != 2 || !a.zero || a.amode != 0 || a.cwrap != 0 || a.ln_g || a.y2 || a.up) return false;
  if (a.Cin % 64 || a.Cout % 8 || a.ldy % 8 || (a.res1 && a.ldr1 % 8) || (a.res2 && a.ldr2 % 8)) return false;
  if (a.x2 && a.C1 < a.Cin) return false;
  const int HWo = a.Ho * a.Wo;
  const bool batched = a.w_bstride > 0;
  return (a.act == ACT_NONE || a.act == ACT_SILU) && (batched || HWo % 64 == 0) && a.Cout % 128 == 0;
}

// Mirrors the EPI_GNA branch of conv_dispatch: 1x1, 16-bit, 64x128 swapped tiles inside one
// image, groups of whole 16-byte vectors (the groupnorm_stats layout), Cin <= 512.
bool conv_gna_ok(const ConvArgs& a, int elem_bytes) {
  if (elem_bytes != 2 || !a.zero || a.amode != 0 || a.cwrap != 0 || a.ln_g || a.lnf_cs || a.y2 || a.up) return false;
  // gna_groups >= 4: the statistics merge reduces tpg = 256 / groups lanes with an xor tree
  // inside one wave (conv_impl.h), so a group may not span two waves.
  if (a.x2 || a.w_bstride || a.Cin % 64 || a.Cin > 512 || a.Cin != a.K || a.gna_groups < 4 || a.gna_groups > 64 ||
      (a.gna_groups & (a.gna_groups - 1)))
    return false;
  if (a.Cin % a.gna_groups || (a.Cin / a.gna_groups) % 8 || 256 % (a.Cin / 8)) return false;
  if (a.Cout % 128 || a.ldy % 8 || (a.res1 && a.ldr1 % 8) || (a.res2 && a.ldr2 % 8)) return false;
  return (a.act == ACT_NONE || a.act == ACT_SILU) && (a.Ho * a.Wo) % 64 == 0;
}

// v6 2-D halo tiles (conv_impl.h conv3h_kernel): 16-bit 3x3 s1 p1, 8-row x 64-column output
// tiles of one image, whole 64-channel N tiles, 32-channel K chunks, buffer-descriptor DMA (one
// row pitch, 31-bit byte offsets), the minimal register epilogue, no fused second output.
bool conv3h_ok(const ConvArgs& a, int elem_bytes) {
  if (elem_bytes != 2 || !a.zero || a.amode != 0 || a.cwrap != 0 || a.w_bstride != 0 || a.y2 || a.ln_g || a.lnf_cs ||
      a.gna_stats || a.ys8 || a.xs8 || a.uph)
    return false;
  if (a.Cin % 32 || (a.C1 < a.Cin && a.C1 % 32) || a.K != 9 * a.Cin || a.Cout % 64 || a.Wo % 64 || a.Ho % 8)
    return false;
  if (!(a.act == ACT_NONE || a.act == ACT_SILU) || a.ldy % 8 || (a.res1 && a.ldr1 % 8) || (a.res2 && a.ldr2 % 8))
    return false;
  if (a.x2 && a.C1 < a.Cin && a.ld2 != a.ld1) return false;       // one row pitch (buffer offsets)
  const size_t LIM = (size_t)1 << 30;
  if ((size_t)a.B * a.Hs * a.Ws * a.ld1 * 2 >= LIM || (size_t)a.Cout * a.K * 2 >= LIM) return false;
  if ((a.ss && (a.ss_ld % 4 || a.Cout % 4 || ((uintptr_t)a.ss & 15))) || ((uintptr_t)a.bias & 15)) return false;
  return true;
}

bool conv_res_fusable(const ConvArgs& a) {
  if (!(a.w2 && a.y2 && a.ldy2 % 8 == 0 && a.bias2 == nullptr && a.Cout % 64 == 0)) return false;
  if (g_conv3_force >= 0 || a.cwrap) return false;
  if ((a.ss && (a.ss_ld % 4 || a.Cout % 4 || ((uintptr_t)a.ss & 15))) || ((uintptr_t)a.bias & 15)) return false;
  const int v = conv_variant(a, 3, 2);
  if (v == 12 || v == 27) return true;            // v4 256x64 tiles, or conv3r (CIN 128)
  if (v != 20 && v != 7 && v != 11) return false;     // 128x64 v4 / v3 candidates only
  const bool kok = (a.C1 >= a.Cin || a.C1 % 32 == 0) && a.Cin % 32 == 0;
  return kok && conv3_rw_host(a, 128) > 0 && conv3_rw_host(a, 128) % 32 == 0;
}

// fp8-output block1 (ConvArgs::ys8): mirrors the two dispatcher branches that take it — the
// weight-stationary 64 -> 64 conv (buffer DMA form) and the fused-res_conv v4 256x64 tiles.
bool conv_q8out_ok(const ConvArgs& a0) {
  ConvArgs a = a0;
  a.ys8 = reinterpret_cast<uint8_t*>(&a);          // (asked before the tensor exists)
  if (a.Cout != 64 || a.ldy != 64 || a.res1 || a.res2 || a.bbias || a.xs8 || g_conv3_force >= 0) return false;
  if (!a.y2) {
    const bool buf = (a.C1 >= a.Cin || !a.x2 || a.ld2 == a.ld1) &&
                     (size_t)a.B * a.Hs * a.Ws * a.ld1 * 2 + a.ld1 * 2 < ((size_t)1 << 31);
    return conv3w_ok(a) && buf;
  }
  return conv_res_fusable(a) && conv_variant(a, 3, 2) == 12;
}

// Row-phase upsample conv (ConvArgs::uph; the caller passes the 4-row phase weights with
// K = 12 Cin): mirrors the dispatcher's uph branch — 16-bit v4 256x64 swapped tiles whose RH
// output rows fit a whole number of row pairs, minimal epilogue, no second output.
bool conv_uph_ok(const ConvArgs& a) {
  if (!a.up || !a.zero || a.amode || a.cwrap || a.w_bstride || a.y2 || a.ys8 || a.xs8 || a.ln_g || a.lnf_cs ||
      a.gna_stats || g_conv3_force >= 0)
    return false;
  if (a.Cout % 64 || a.Cin % 64 || (a.C1 < a.Cin && a.C1 % 32) || a.K != (a.uph == 2 ? 16 : 12) * a.Cin) return false;
  if (!(a.act == ACT_NONE || a.act == ACT_SILU) || a.ldy % 8 || (a.res1 && a.ldr1 % 8) || (a.res2 && a.ldr2 % 8))
    return false;
  if ((a.ss && (a.ss_ld % 4 || a.Cout % 4 || ((uintptr_t)a.ss & 15))) || ((uintptr_t)a.bias & 15)) return false;
  const int RW = conv3_rw_host(a, 256);
  return RW > 0 && RW % 64 == 0 && a.Ho % (2 * (256 / RW)) == 0 && (a.uph != 2 || RW >= 128);
}

// Split-K for 1x1 GEMMs whose 64x128 tile grid covers under half the CUs (the ViT and text
// tower linears at M = B x L rows): enough K splits to fill the chip, each with >= 4 K tiles.
// The split count is a function of `rows` = ONE image's rows (L), never of the batch: the
// partial sums' order then does not depend on what else is in the batch, so an image's result
// is bit-identical in any batch / shard. 0 = no split. Plain epilogues only (no row LayerNorm,
// folds, GEGLU or per-image weights).
int conv_split_k(const ConvArgs& a, int elem_bytes, long rows) {
  if (a.ln_g || a.lnf_cs || a.gna_stats || a.w_bstride || a.act == ACT_GEGLU || a.amode || a.cwrap || a.up ||
      a.ys8 || a.xs8 || a.uph || !a.zero || a.Cin != a.K || a.Cout < 64)
    return 0;
  if (getenv("DAC_SPLITK") && atoi(getenv("DAC_SPLITK")) == 0) return 0;
  const int BKE = 128 / elem_bytes;
  if (a.K % BKE) return 0;
  if (rows <= 0) return 0;
  const long tiles = ((rows + 63) / 64) * ((a.Cout + 127) / 128);
  const int nk = a.K / BKE;
  if (tiles >= 128 || nk < 8) return 0;
  int s = (int)((256 + tiles - 1) / tiles);
  s = s > nk / 4 ? nk / 4 : s;
  s = s > 8 ? 8 : s;
  return s >= 2 ? s : 0;
}

bool conv3_split_ok(const ConvArgs& a, int elem_bytes) {
  const int VEh = 16 / elem_bytes, BKE = 128 / elem_bytes;
  if (a.y2 || a.w2 || a.up || a.uph || a.ys8 || a.xs8 || a.cwrap || a.w_bstride || a.amode || a.ln_g ||
      a.lnf_cs || a.gna_stats || !a.zero)
    return false;
  if (a.act != ACT_NONE && a.act != ACT_SILU) return false;
  if (a.Cin % BKE || a.Cout % VEh || a.ldy % VEh || a.Cout <= 16) return false;
  if (a.Ho != a.Hs || a.Wo != a.Ws || a.K != 9 * a.Cin) return false;
  if (a.x2 && a.C1 % BKE) return false;
  return conv3_rw_host(a, 128) > 0 && conv3_rw_host(a, 256) > 0;
}

int conv3_split_k(const ConvArgs& a, int elem_bytes, int ks) {
  if (ks < 2 || !conv3_split_ok(a, elem_bytes)) return 0;
  const int nchunk = a.Cin / (128 / elem_bytes);
  while (ks > 1 && nchunk / ks < 2) --ks;
  return ks >= 2 ? ks : 0;
}

template <typename T>
__global__ void __launch_bounds__(256) conv_part_reduce_kernel(ConvArgs a, int M, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % a.Cout);
  const int m = (int)(i / a.Cout);
  float v = 0.f;
  for (int z = 0; z < a.ksplit; ++z) v += a.part[((size_t)z * M + m) * a.Cout + c];
  const int HWo = a.Ho * a.Wo, b = m / HWo;
  // The register epilogues' fast path: bias folded into the shift, SiLU in the log2 domain.
  float s = 1.f, h = 0.f;
  if (a.ss) { s += a.ss[(size_t)b * a.ss_ld + c]; h = a.ss[(size_t)b * a.ss_ld + a.Cout + c]; }
  const bool silu = a.act == ACT_SILU;
  epi_fold(a.bias ? a.bias[c] : 0.f, s, h, silu);
  v = fmaf(v, s, h);
  if (silu) v = silu_log2(v);
  else if (a.act == ACT_GELU) v = gelu_fast(v);
  if (a.res1) v += to_f(reinterpret_cast<const T*>(a.res1)[(size_t)m * a.ldr1 + c]);
  if (a.res2) v += to_f(reinterpret_cast<const T*>(a.res2)[(size_t)m * a.ldr2 + c]);
  if (a.bbias) v += a.bbias[(size_t)b * a.bb_ld + c];
  reinterpret_cast<T*>(a.y)[(size_t)m * a.ldy + c] = from_f<T>(v);
}

template <typename T>
void conv_part_reduce(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.Ho * a.Wo;
  const size_t n = (size_t)M * a.Cout;
  conv_part_reduce_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, M, n);
}
template void conv_part_reduce<float>(const ConvArgs&, hipStream_t);
template void conv_part_reduce<bf16>(const ConvArgs&, hipStream_t);
template void conv_part_reduce<f16>(const ConvArgs&, hipStream_t);

template <typename T>
void conv(const ConvArgs& a, int kh, int kw, int s, int p, hipStream_t st) {
  if (a.xs8) throw std::invalid_argument("conv: e4m3 inputs are conv3q-only");
  if (kh == 3 && kw == 3 && s == 1 && p == 1) conv_dispatch<T, 3, 3, 1, 1>(a, st);
  else if (kh == 1 && kw == 1 && s == 1 && p == 0) conv_dispatch<T, 1, 1, 1, 0>(a, st);
  else if (kh == 4 && kw == 4 && s == 2 && p == 1) conv_dispatch<T, 4, 4, 2, 1>(a, st);
  else if (kh == 7 && kw == 7 && s == 1 && p == 3) conv_dispatch<T, 7, 7, 1, 3>(a, st);
  else if (kh == 32 && kw == 32 && s == 32 && p == 0) conv_dispatch<T, 32, 32, 32, 0>(a, st);
  else if (kh == 14 && kw == 14 && s == 14 && p == 0) conv_dispatch<T, 14, 14, 14, 0>(a, st);
  else throw std::invalid_argument("conv: unsupported kernel/stride/padding");
}

template void conv<float>(const ConvArgs&, int, int, int, int, hipStream_t);
template void conv<bf16>(const ConvArgs&, int, int, int, int, hipStream_t);
template void conv<f16>(const ConvArgs&, int, int, int, int, hipStream_t);

}  // namespace dac
