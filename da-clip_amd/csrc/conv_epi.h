// conv_epi.h — shared epilogue of the implicit-GEMM conv kernels.
//
// Phase 1 (registers): bias -> per-image scale/shift -> SiLU/GELU (or the GEGLU pairing of
// accumulator tiles j, j+1) on each wave's TM x TN 16x16 accumulators, written as fp32 into
// an LDS image of the block tile [BM][BN] (row pad 16 B: the 4 lane groups of a wave land on
// disjoint bank quarters).
// Phase 2 (coalesced): every thread moves 16-byte output chunks (VE channels of one row):
// + res1 + res2 + per-image bias, one 16-byte store; rows map through `rowmap` (row-halo
// tiles are 2-D in the image). Partial / misaligned chunks fall back to scalars.
// Keeping the LDS image in fp32 keeps the residual adds in fp32 like the reference.
// The tile goes through LDS in BM / EPR passes of EPR rows (EPR a multiple of the wave row
// height), so the epilogue never needs more LDS than the main loop's pipeline: the kernels
// pick EPR to keep several blocks resident per CU.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dac {

struct LinearRows {      // block-tile row t -> output row m0 + t
  int m0;
  DEV int operator()(int t) const { return m0 + t; }
};

template <typename T> DEV float silu_t(float x);
template <> DEV float silu_t<float>(float x) { return x / (1.f + expf(-x)); }
// 16-bit outputs: v_rcp_f32 (1 ulp) instead of a correctly rounded reciprocal, which compiles
// to the ~10-instruction IEEE division sequence and dominated the SiLU epilogues.
template <> DEV float silu_t<bf16>(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
template <> DEV float silu_t<f16>(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// 16-bit epilogues fold the per-channel terms once: u = (acc + b) * s + h = acc * s + (b * s + h),
// and with SiLU they also carry log2(e) in (s, h), so u2 = u * log2(e) comes out of the same fma,
// 2^-u2 = e^-u needs no extra multiply and silu(u) = u2 * rcp(fma(2^-u2, log2e, log2e)): three
// VALU + v_exp + v_rcp per value instead of five + the two. Every epilogue path of a kernel uses
// the same fold, so a row rounds identically whichever path its tile takes (batch invariance).
constexpr float kL2E = 1.4426950408889634f;
DEV void epi_fold(float b, float& s, float& h, bool silu) {
  h = fmaf(b, s, h);
  if (silu) { s *= kL2E; h *= kL2E; }
}
DEV float silu_log2(float u2) { return u2 * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(-u2), kL2E, kL2E)); }

template <int BM, int BN>
struct EpiLds {
  static constexpr int LDW = BN + 4;                 // floats per LDS row
  static constexpr int BYTES = BM * LDW * 4;
};

// Largest pass height (multiple of WTM dividing BM) whose fp32 tile fits in `budget` bytes;
// WTM if none does (the caller then sizes LDS for that).
template <int BM, int BN, int WTM>
constexpr int epi_rows(int budget) {
  int best = WTM;
  for (int r = WTM; r <= BM; r += WTM)
    if (BM % r == 0 && EpiLds<1, BN>::LDW * 4 * r <= budget) best = r;
  return best;
}

// Epilogue feature set compiled into a kernel (EPK bits). A kernel that can only meet the
// fast case (tile inside one image, SiLU / none, 16-byte aligned rows) compiles EPI_MIN and
// stays small: the epilogue runs once per block, and every path compiled into it costs
// instruction-cache fetches on that one pass.
enum : int { EPI_GENERAL = 1, EPI_GEGLU = 2, EPI_GELU = 4, EPI_SCALAR = 8, EPI_MIN = 0, EPI_ALL = 15,
             EPI_LN = 16, EPI_SWAP = 32,   // EPI_SWAP: swapped operands + epi_regs16 (conv_impl.h)
             EPI_LNF = 64,                 // input LayerNorm folded into a 1x1 GEMM (ConvArgs::lnf_cs)
             EPI_GNA = 128,                // input GroupNorm applied in the A path (ConvArgs::gna_stats)
             EPI_PART = 256 };             // split-K partial sums to ConvArgs::part (no epilogue)

// Per-channel epilogue terms of this lane's accumulator columns (bias, 1 + scale, shift) for a
// tile inside image bimg; kernels that know bimg up front load them before the main loop.
template <int TN> struct EpiTerms { float bi[TN], sc[TN], sh[TN]; };

template <int TN>
DEV EpiTerms<TN> epi_terms(const ConvArgs& a, int n0, int bimg, int colbase) {
  EpiTerms<TN> e;
  const int lr = threadIdx.x & 15;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + colbase + j * 16 + lr;
    const bool ok = n < a.Cout;
    e.bi[j] = (a.bias && ok) ? a.bias[n] : 0.f;
    e.sc[j] = 1.f; e.sh[j] = 0.f;
    if (a.ss && ok) {
      const float* s = a.ss + (size_t)bimg * a.ss_ld;
      e.sc[j] = s[n] + 1.f;
      e.sh[j] = s[a.Cout + n];
    }
  }
  return e;
}

// ILV > 1: accumulator tile i, row m of a wave holds wave pixel m * ILV + i (the interleaved
// row order of conv3i_kernel); ILV = 1 is the plain order i * 16 + m.
template <typename T, int BM, int BN, int WGM, int WGN, int EPR, int EPK = EPI_ALL, int ILV = 1,
          class RowMap>
DEV void conv_epilogue_lds(const ConvArgs& a, f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16],
                           char* smem, int M, const RowMap& rowmap, int n0, int HWo, int bimg,
                           const EpiTerms<BN / WGN / 16>* pre = nullptr) {
  constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 16, TN = WTN / 16;
  static_assert(EPR % WTM == 0 && BM % EPR == 0, "epilogue pass height");
  static_assert(ILV == 1 || ILV == TM, "interleave = tiles per wave");
  // Wave-relative row of accumulator element (tile i, lane group lg, register r).
  auto arow = [](int i, int lg, int r) { return ILV == 1 ? i * 16 + lg * 4 + r : (lg * 4 + r) * ILV + i; };
  constexpr int NT = 64 * WGM * WGN;
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int LDW = EpiLds<BM, BN>::LDW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int lr = lane & 15, lg = lane >> 4;
  // EPK == EPI_GEGLU kernels are launched for GEGLU only: compile only that path (the runtime
  // choice kept the other one live and pushed the accumulators to scratch).
  constexpr bool GEGLU_ONLY = EPK == EPI_GEGLU;
  const bool geglu = GEGLU_ONLY || ((EPK & EPI_GEGLU) && a.act == ACT_GEGLU);
  const bool fast = !(EPK & EPI_GENERAL) || bimg >= 0;
  float* tile = reinterpret_cast<float*>(smem);

  T* y = reinterpret_cast<T*>(a.y);
  const T* r1 = reinterpret_cast<const T*>(a.res1);
  const T* r2 = reinterpret_cast<const T*>(a.res2);
  // EPI_MIN kernels (single pass, vector rows): issue this thread's residual loads first, so
  // their latency overlaps the accumulator math and LDS staging below.
  constexpr bool PREF = EPK == EPI_MIN && EPR == BM;     // (EPI_LN kernels take their own path)
  constexpr int CPRF = BN / VE;
  constexpr int NKP = PREF ? (BM * CPRF + NT - 1) / NT : 1;
  u32x4 rv1[NKP], rv2[NKP];
  if constexpr (PREF) {
#pragma unroll
    for (int k = 0; k < NKP; ++k) {
      const int c = tid + k * NT;
      const int m = rowmap(c / CPRF), n = n0 + (c % CPRF) * VE;
      const bool ok = c < BM * CPRF && m < M && n < a.Cout;
      rv1[k] = (r1 && ok) ? *reinterpret_cast<const u32x4*>(r1 + (size_t)m * a.ldr1 + n) : u32x4{0u, 0u, 0u, 0u};
      rv2[k] = (r2 && ok) ? *reinterpret_cast<const u32x4*>(r2 + (size_t)m * a.ldr2 + n) : u32x4{0u, 0u, 0u, 0u};
    }
  }

  // Fast path: all rows of the tile belong to image bimg -> per-channel terms in registers.
  EpiTerms<TN> et;
  if (pre) et = *pre;
  else if (fast) et = epi_terms<TN>(a, n0, bimg, wn * WTN);
  else {
#pragma unroll
    for (int j = 0; j < TN; ++j) { et.bi[j] = 0.f; et.sc[j] = 1.f; et.sh[j] = 0.f; }
  }
  const float* bi = et.bi;
  const float* sc = et.sc;
  const float* sh = et.sh;
  const bool vec_ok = (a.ldy % VE == 0) && (!r1 || a.ldr1 % VE == 0) && (!r2 || a.ldr2 % VE == 0);
  // Prefetched variant (PREF): chunk k of this thread.
  auto emit_pre = [&](int k, int t, const float* src, int n) __attribute__((always_inline)) {
    const int m = rowmap(t);
    if (m >= M || n >= a.Cout) return;
    float v[VE];
#pragma unroll
    for (int e = 0; e < VE; e += 4) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(src + e);
      v[e] = q[0]; v[e + 1] = q[1]; v[e + 2] = q[2]; v[e + 3] = q[3];
    }
    const T* e1 = reinterpret_cast<const T*>(&rv1[k]);
    const T* e2 = reinterpret_cast<const T*>(&rv2[k]);
    if (r1) {
#pragma unroll
      for (int e = 0; e < VE; ++e) v[e] += to_f(e1[e]);
    }
    if (r2) {
#pragma unroll
      for (int e = 0; e < VE; ++e) v[e] += to_f(e2[e]);
    }
    if (a.bbias) {
      const float* bb = a.bbias + (size_t)bimg * a.bb_ld + n;
#pragma unroll
      for (int e = 0; e < VE; ++e) v[e] += bb[e];
    }
    store_vec<T>(y + (size_t)m * a.ldy + n, v);
  };
  // t: tile row, src: its LDS row.
  auto emit = [&](int t, const float* src, int n, int Cout) __attribute__((always_inline)) {
    const int m = rowmap(t);
    if (m >= M || n >= Cout) return;
    float v[VE];
#pragma unroll
    for (int e = 0; e < VE; e += 4) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(src + e);
      v[e] = q[0]; v[e + 1] = q[1]; v[e + 2] = q[2]; v[e + 3] = q[3];
    }
    const int b = bimg >= 0 ? bimg : m / HWo;
    if (!(EPK & EPI_SCALAR) || (vec_ok && n + VE <= Cout)) {
      float t1[VE];
      if (r1) {
        load_vec<T>(r1 + (size_t)m * a.ldr1 + n, t1);
#pragma unroll
        for (int e = 0; e < VE; ++e) v[e] += t1[e];
      }
      if (r2) {
        load_vec<T>(r2 + (size_t)m * a.ldr2 + n, t1);
#pragma unroll
        for (int e = 0; e < VE; ++e) v[e] += t1[e];
      }
      if (a.bbias) {
        const float* bb = a.bbias + (size_t)b * a.bb_ld + n;
#pragma unroll
        for (int e = 0; e < VE; ++e) v[e] += bb[e];
      }
      store_vec<T>(y + (size_t)m * a.ldy + n, v);
    } else if constexpr ((EPK & EPI_SCALAR) != 0) {
      for (int e = 0; e < VE && n + e < Cout; ++e) {
        float u = v[e];
        if (r1) u += to_f(r1[(size_t)m * a.ldr1 + n + e]);
        if (r2) u += to_f(r2[(size_t)m * a.ldr2 + n + e]);
        if (a.bbias) u += a.bbias[(size_t)b * a.bb_ld + n + e];
        y[(size_t)m * a.ldy + n + e] = from_f<T>(u);
      }
    }
  };

  // Phase 1a, once: bias -> scale/shift -> activation (GEGLU: x * gelu(gate) into the even
  // tile) in place on the accumulators. Doing it before the pass loop keeps the (speculated)
  // math out of the per-pass guarded stores.
  if (fast && geglu) {
    // GEGLU (no scale/shift): x tile j, gate tile j+1, biases from the preloaded terms.
    if constexpr (TN % 2 == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j2 = 0; j2 < TN / 2; ++j2)
            acc[i][2 * j2][r] = (acc[i][2 * j2][r] + bi[2 * j2]) * gelu_fast(acc[i][2 * j2 + 1][r] + bi[2 * j2 + 1]);
    }
  } else if (!GEGLU_ONLY && fast) {
    if constexpr (sizeof(T) == 2) {
      // Folded terms (epi_fold), SiLU in the log2 domain; the general path below folds alike.
      const bool silu = a.act == ACT_SILU;
      float fs[TN], fh[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) { fs[j] = sc[j]; fh[j] = sh[j]; epi_fold(bi[j], fs[j], fh[j], silu); }
      if (silu) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j][r] = silu_log2(fmaf(acc[i][j][r], fs[j], fh[j]));
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              float v = fmaf(acc[i][j][r], fs[j], fh[j]);
              if ((EPK & EPI_GELU) && a.act == ACT_GELU) v = gelu_fast(v);
              acc[i][j][r] = v;
            }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            // Explicit fma (and in the general path below): both paths round identically, so a
            // row's result does not depend on whether its tile spans images (batch invariance).
            float v = fmaf(acc[i][j][r] + bi[j], sc[j], sh[j]);
            if (a.act == ACT_SILU) v = silu_t<T>(v);
            else if ((EPK & EPI_GELU) && a.act == ACT_GELU) v = gelu_fast(v);
            acc[i][j][r] = v;
          }
    }
  } else if constexpr ((EPK & EPI_GENERAL) != 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = wm * WTM + arow(i, lg, r);
        if (geglu) {
          if constexpr (TN % 2 == 0) {
#pragma unroll
            for (int j = 0; j < TN; j += 2) {
              const int nx = n0 + wn * WTN + j * 16 + lr;
              float vx = acc[i][j][r], vg = acc[i][j + 1][r];
              if (a.bias && nx < a.Cout) { vx += a.bias[nx]; vg += a.bias[nx + 16]; }
              acc[i][j][r] = vx * gelu_fast(vg);
            }
          }
          continue;
        }
        const int m = rowmap(t);
        const int b = bimg >= 0 ? bimg : (m < M ? m / HWo : 0);
        const float* s = a.ss ? a.ss + (size_t)b * a.ss_ld : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WTN + j * 16 + lr;
          float v = acc[i][j][r];
          if constexpr (sizeof(T) == 2) {
            // The fast path's fold, element by element (identical rounding).
            const bool silu = a.act == ACT_SILU;
            float fs = 1.f, fh = 0.f, fb = 0.f;
            if (n < a.Cout) {
              if (a.bias) fb = a.bias[n];
              if (s) { fs = s[n] + 1.f; fh = s[a.Cout + n]; }
            }
            epi_fold(fb, fs, fh, silu);
            v = fmaf(v, fs, fh);
            if (silu) v = silu_log2(v);
            else if ((EPK & EPI_GELU) && a.act == ACT_GELU) v = gelu_fast(v);
          } else {
            if (n < a.Cout) {
              if (a.bias) v += a.bias[n];
              if (s) v = fmaf(v, s[n] + 1.f, s[a.Cout + n]);
            }
            if (a.act == ACT_SILU) v = silu_t<T>(v);
            else if ((EPK & EPI_GELU) && a.act == ACT_GELU) v = gelu_fast(v);
          }
          acc[i][j][r] = v;
        }
      }
    }
  }

#pragma unroll
  for (int r0 = 0; r0 < BM; r0 += EPR) {
    __syncthreads();                                 // main-loop / previous-pass LDS reads done
    // Phase 1b: the waves whose rows fall in this pass store them (fp32) to the LDS tile.
    if (wm * WTM >= r0 && wm * WTM < r0 + EPR) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* row = tile + (wm * WTM - r0 + arow(i, lg, r)) * LDW;
          if (geglu) {
            if constexpr (TN % 2 == 0) {
#pragma unroll
              for (int j2 = 0; j2 < TN / 2; ++j2) row[(wn * WTN + j2 * 32) / 2 + lr] = acc[i][2 * j2][r];
            }
          } else if constexpr (!GEGLU_ONLY) {
#pragma unroll
            for (int j = 0; j < TN; ++j) row[wn * WTN + j * 16 + lr] = acc[i][j][r];
          }
        }
    }
    __syncthreads();
    const int CPR = geglu ? BN / 2 / VE : BN / VE;   // 16-byte chunks per tile row
    const int nch = EPR * CPR;
    if constexpr ((EPK & EPI_LN) != 0) {
      // Row LayerNorm over the BN (= Cout) channels of each tile row: the CPR threads of a row
      // are consecutive lanes, so mean and variance are two xor-shuffle reductions (two-pass,
      // every lane takes part: (EPR * CPR) % NT == 0 is checked at compile time).
      static_assert((EPR * (BN / VE)) % NT == 0 && (BN / VE) <= 64, "LN epilogue tiling");
#pragma unroll
      for (int k = 0; k < EPR * (BN / VE) / NT; ++k) {
        const int c = tid + k * NT;
        const int tl = c / CPR, cc = (c % CPR) * VE;
        const float* src = tile + tl * LDW + cc;
        float v[VE];
#pragma unroll
        for (int e = 0; e < VE; e += 4) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(src + e);
          v[e] = q[0]; v[e + 1] = q[1]; v[e + 2] = q[2]; v[e + 3] = q[3];
        }
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < VE; ++e) s += v[e];
#pragma unroll
        for (int o = 1; o < BN / VE; o <<= 1) s += __shfl_xor(s, o, 64);
        const float mean = s / (float)BN;
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < VE; ++e) { const float d = v[e] - mean; q += d * d; }
#pragma unroll
        for (int o = 1; o < BN / VE; o <<= 1) q += __shfl_xor(q, o, 64);
        const float rstd = 1.f / sqrtf(q / (float)BN + a.ln_eps);
        const int m = rowmap(r0 + tl), n = n0 + cc;
        if (m < M) {
#pragma unroll
          for (int e = 0; e < VE; ++e) v[e] = (v[e] - mean) * rstd * a.ln_g[n + e];
          float t1[VE];
          if (r1) {
            load_vec<T>(r1 + (size_t)m * a.ldr1 + n, t1);
#pragma unroll
            for (int e = 0; e < VE; ++e) v[e] += t1[e];
          }
          store_vec<T>(y + (size_t)m * a.ldy + n, v);
        }
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < (EPR * (BN / VE) + NT - 1) / NT; ++k) {
      const int c = tid + k * NT;
      if (c >= nch) break;
      const int tl = c / CPR, cc = (c % CPR) * VE;
      if constexpr (PREF) emit_pre(k, tl, tile + tl * LDW + cc, n0 + cc);
      else if (geglu) emit(r0 + tl, tile + tl * LDW + cc, n0 / 2 + cc, a.Cout / 2);
      else emit(r0 + tl, tile + tl * LDW + cc, n0 + cc, a.Cout);
    }
  }
}

}  // namespace dac
