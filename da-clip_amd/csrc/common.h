// common.h — shared device helpers for the gfx950 kernels of libdaclip_hip.
//
// Storage/compute types: `float` (parity mode, exact-f32 MFMA v_mfma_f32_16x16x4_f32),
// `bf16` (perf mode, v_mfma_f32_16x16x32_bf16, fp32 accumulate) and `f16` (IEEE half, same
// shapes on v_mfma_f32_16x16x32_f16). Every tile operand is read from LDS as one 16-byte
// vector per lane, so one kernel body serves all types: a 16-byte vector holds
// VE = 16/sizeof(T) elements (8 bf16 / f16 or 4 f32).
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <stdint.h>

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

// 16-bit storage types: bf16 (8-bit significand, the configs[1] perf mode) and IEEE fp16
// (11-bit significand: 8x less rounding error at the same bytes and the same MFMA rate; the
// mode that holds the 1e-3 dB PSNR bar). Both use 8 elements per 16-byte vector.
template <typename T> struct TypeInfo;
template <> struct TypeInfo<float> { static constexpr int VE = 4; };
template <> struct TypeInfo<bf16> { static constexpr int VE = 8; };
template <> struct TypeInfo<f16> { static constexpr int VE = 8; };
template <typename T> struct Vec8;
template <> struct Vec8<bf16> { typedef bf16x8 t; typedef bf16x2_t t2; };
template <> struct Vec8<f16> { typedef f16x8 t; typedef f16x2_t t2; };

DEV float to_f(float v) { return v; }
DEV float to_f(bf16 v) { return (float)v; }
DEV float to_f(f16 v) { return (float)v; }
template <typename T> DEV T from_f(float v);
template <> DEV float from_f<float>(float v) { return v; }
template <> DEV bf16 from_f<bf16>(float v) { return (bf16)v; }
template <> DEV f16 from_f<f16>(float v) { return (f16)v; }

// Two packed 16-bit elements (low half first) -> two floats. bf16 by bit shifts (no
// conversion instruction, no spills), fp16 by v_cvt_f32_f16.
template <typename T> DEV void unpack2(unsigned u, float& lo, float& hi);
template <> DEV void unpack2<bf16>(unsigned u, float& lo, float& hi) {
  lo = __uint_as_float(u << 16);
  hi = __uint_as_float(u & 0xffff0000u);
}
template <> DEV void unpack2<f16>(unsigned u, float& lo, float& hi) {
  const f16x2_t h = __builtin_bit_cast(f16x2_t, u);
  lo = (float)h[0];
  hi = (float)h[1];
}

// lo += element 0, hi += element 1 of a packed pair (a residual added to fp32 epilogue values).
// fp16: one v_fma_mix_f32 per element (the half is converted inside the fma: r * 1 + v, the same
// single rounding as convert + add) instead of a v_cvt_f32_f16 and a v_add_f32.
template <typename T> DEV void add_pair(unsigned u, float& lo, float& hi) {
  float a, b;
  unpack2<T>(u, a, b);
  lo += a;
  hi += b;
}
template <> DEV void add_pair<f16>(unsigned u, float& lo, float& hi) {
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(u));
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(hi) : "v"(u));
}

// Load / store VE elements (16 bytes) as fp32 values.
template <typename T> DEV void load_vec(const T* p, float* out);
template <> DEV void load_vec<float>(const float* p, float* out) {
  f32x4 v = *reinterpret_cast<const f32x4*>(p);
  out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
}
template <> DEV void load_vec<bf16>(const bf16* p, float* out) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = (float)v[i];
}
template <> DEV void load_vec<f16>(const f16* p, float* out) {
  f16x8 v = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = (float)v[i];
}
template <typename T> DEV void store_vec(T* p, const float* in);
template <> DEV void store_vec<float>(float* p, const float* in) {
  *reinterpret_cast<f32x4*>(p) = f32x4{in[0], in[1], in[2], in[3]};
}
template <> DEV void store_vec<bf16>(bf16* p, const float* in) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)in[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}
template <> DEV void store_vec<f16>(f16* p, const float* in) {
  f16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (f16)in[i];
  *reinterpret_cast<f16x8*>(p) = v;
}

// ---------------------------------------------------------------------------------------
// MFMA 16x16 tile step. acc(16x16) += A(16 x KSTEP) * B(KSTEP x 16), where lane l supplies
// 16 bytes of row (l&15) of A (resp. column (l&15) of B stored n-major) at k-offset
// KSTEP/4 * (l>>4) elements. For bf16 one v_mfma_f32_16x16x32_bf16 consumes the vector.
// For f32 the 4 floats feed 4 v_mfma_f32_16x16x4_f32 (element j of lane group g is
// k = 4g + j): any k-permutation shared by A and B leaves the sum unchanged, so the result
// is an exact-f32 dot product over the same 16 k values.
// C layout (both): acc[r] = C[row = 4*(l>>4) + r][col = l&15].
template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KSTEP = 32;
  DEV static void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<f16> {
  static constexpr int KSTEP = 32;
  DEV static void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                 __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KSTEP = 16;
  DEV static void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
  }
};

// Kernel arguments live in a fresh kernarg buffer per launch, so the first scalar load of every
// 64-byte line of it misses the scalar cache. hipcc loads a struct argument's fields lazily, each
// group behind its own s_waitcnt: a ConvArgs kernel paid five dependent misses (~1.2 us of its
// prologue, tools/convbench_stamp). Touching every line once, up front, behind ONE wait turns the
// later loads into hits.
typedef const volatile __attribute__((address_space(4))) uint32_t kernarg_u32;
template <int BYTES> DEV void kernarg_touch() {
  kernarg_u32* p = (kernarg_u32*)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t acc = 0;
#pragma unroll
  for (int o = 0; o < BYTES; o += 64) acc ^= p[o / 4];
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(acc) : "memory");
}

// In-graph launch timing (engine Profiler::stamps; HIP events cannot be timed inside graph
// replays): a kernel declares `StampGuard sg(a.stamp);` first thing. With a non-null stamp
// block (STAMP_SLOTS [begin, end] pairs of 64-bit words per launch) the first wave of every
// block atomic-mins the wall clock into its slot's begin and, on every exit path, each wave
// atomic-maxes the clock into the slot's end; the slot is blockIdx.x % STAMP_SLOTS, which spreads
// the atomics over 64 addresses (one address for a whole grid serialised them and stretched the
// profiled replay by a fifth). min(begin) .. max(end) over a launch's slots is its duration on the
// constant-rate counter (s_memrealtime, 100 MHz; ticks to ms by hipDeviceAttributeWallClockRate).
// Null (every production launch): one uniform branch.
constexpr int STAMP_SLOTS = 64;
struct StampGuard {
  unsigned long long* s;
  DEV explicit StampGuard(unsigned long long* p) : s(p ? p + 2 * (blockIdx.x % STAMP_SLOTS) : nullptr) {
    if (s && threadIdx.x == 0) atomicMin(s, (unsigned long long)wall_clock64());
  }
  DEV ~StampGuard() {
    if (s && (threadIdx.x & 63) == 0) atomicMax(s + 1, (unsigned long long)wall_clock64());
  }
};

DEV float silu_f(float x) { return x / (1.f + expf(-x)); }
DEV float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
// Exact-form GELU 0.5 x (1 + erf(x / sqrt 2)) with erf from Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7): 1 + erf is formed as 2 - q or q, q = erfc(|z|) = t P(t) exp(-z^2), so
// the negative tail has no cancellation. About 12 instructions against ~30 for erff; used by
// the GEMM epilogues (GEGLU, ViT MLP), where erff dominated the epilogue.
DEV float gelu_fast(float x) {
  // No FP contraction: the value must not depend on the inlining context (an epilogue's fast
  // and general paths must agree bit for bit, or results depend on batch composition).
#pragma clang fp contract(off)
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));   // v_rcp_f32, 1 ulp
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                                   -0.284496736f), 0.254829592f);
  const float q = p * __expf(-z * z);
  return 0.5f * x * (x >= 0.f ? 2.f - q : q);
}

// Cross-row reductions on the VALU (gfx950 v_permlane16/32_swap): swapping a register pair
// that both hold x leaves {x, partner} in the pair (in some order), so combining the two gives
// x (op) x^16 or x (op) x^32 in every lane -- the same values as __shfl_xor, without an
// LDS-crossbar round trip and its lgkmcnt wait. Inline asm: the compiler folds the builtin's
// two results into one when both inputs are the same value (it then combined x with itself);
// the s_nop 1 covers the VALU-write -> permlane-read hazard the asm hides from the compiler.
DEV void perm16_swap(float& a, float& b) { asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }
DEV void perm32_swap(float& a, float& b) { asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }
DEV float red16_sum(float v) { float a = v, b = v; perm16_swap(a, b); return a + b; }
DEV float red32_sum(float v) { float a = v, b = v; perm32_swap(a, b); return a + b; }
// The max is taken inside the asm too: an fmaxf on asm outputs makes the compiler canonicalize
// both operands first (two extra v_max x,x); the inputs here are already canonical values.
DEV float red16_max(float v) {
  float a = v, b = v;
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_max_f32 %0, %0, %1" : "+v"(a), "+v"(b));
  return a;
}
DEV float red32_max(float v) {
  float a = v, b = v;
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_max_f32 %0, %0, %1" : "+v"(a), "+v"(b));
  return a;
}
// max of three without the operand canonicalization fmaxf gets on values the compiler cannot
// prove canonical (MFMA accumulators): one v_max3_f32 instead of up to five instructions.
DEV float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
