// attn.hip — self-attention kernels.
//
// flash_attn_d32: SpatialTransformer self-attention (attention.py:170-193: heads = C/32,
// d_head = 32, L = (H/8)*(W/8) tokens). Flash-style, one workgroup = 64 (or 128) queries of one
// (image, head), 4 waves x 16 queries, key tiles of 64 through LDS, online softmax in fp32.
// Computed transposed: S^T = K Q^T (A = K rows from LDS, B = this wave's 16 queries held in
// registers) and O^T = V^T P^T. Because the S^T accumulator keeps keys in registers and
// queries on lanes, P^T feeds the second MFMA straight from registers: the k order inside a
// step is permuted identically for V^T (read from LDS in that order), so no LDS round trip
// for P is needed.
//
// small_mha: nn.MultiheadAttention core of the ViT blocks (transformer.py:203, 217-230):
// L = 50 (B/32) tokens, 12 heads x 64; tiny, one workgroup per (image, head), fp32 math.
#include "common.h"

#include <atomic>
#include "kernels.h"
#include <cstdlib>

namespace dac {

// 1: always the staged-tile kernel (DAC_FLASH_OLD=1, or dac_op_attention variant 1).
int g_flash_old = getenv("DAC_FLASH_OLD") ? atoi(getenv("DAC_FLASH_OLD")) : 0;

template <typename T, int QG>
__global__ void __launch_bounds__(256) flash_d32_kernel(const T* __restrict__ qkv, T* o, int L,
                                                        int H, float scale) {
  constexpr int D = 32;
  constexpr int KT = 64;                     // keys per tile
  constexpr int ES = sizeof(T);
  constexpr int KROW = D * ES + 16;          // padded K row (bytes)
  constexpr int VROW = KT * ES + 16;         // padded V^T row (bytes)
  constexpr int KSTEP = Mma<T>::KSTEP;
  __shared__ __attribute__((aligned(16))) char sK[KT * KROW];
  __shared__ __attribute__((aligned(16))) char sV[D * VROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // XCD-aware block order: the dispatcher deals consecutive blocks to the 8 XCDs in turn, so
  // the query tiles of one (image, head) would load its K / V into 8 different L2s. Map each
  // XCD to a contiguous range of (query tile fastest, head, image) instead.
  const int gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xq = n / 8, xr = n % 8, xcd = id % 8;
  const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + id / 8;
  const int bx = t % gx, h = (t / gx) % gy, b = t / (gx * gy);
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;
  // QG groups of 16 queries per wave: every staged K/V tile and K fragment serves all of them.
  int qi[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) qi[g] = bx * (64 * QG) + wave * (16 * QG) + g * 16 + lr;

  // Q fragments (B operand of S^T = K Q^T): column = query, k = d.
  u32x4 qf[QG][D / KSTEP];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int s = 0; s < D / KSTEP; ++s) {
      const int d0 = s * KSTEP + lg * (KSTEP / 4);
      qf[g][s] = qi[g] < L ? *reinterpret_cast<const u32x4*>(base + (size_t)qi[g] * ld + h * D + d0)
                           : u32x4{0u, 0u, 0u, 0u};
    }

  f32x4 oacc[QG][2];
  float mrun[QG], lrun[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    oacc[g][0] = oacc[g][1] = f32x4{0, 0, 0, 0};
    mrun[g] = -INFINITY; lrun[g] = 0.f;
  }
  constexpr int VE = TypeInfo<T>::VE;
  constexpr int NVEC = KT * D / VE;          // 16-byte vectors per K (or V) tile

  // K / V of the next key tile are loaded into registers while this tile computes.
  constexpr int NPT = NVEC / 256;            // vectors per thread per tile
  static_assert(NVEC % 256 == 0, "tile");
  u32x4 kreg[NPT], vreg[NPT];
  auto kv_load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int v = tid + j * 256;
      const int key = v / (D / VE), dv = (v % (D / VE)) * VE;
      const int kk = k0 + key;
      kreg[j] = vreg[j] = u32x4{0u, 0u, 0u, 0u};
      if (kk < L) {
        kreg[j] = *reinterpret_cast<const u32x4*>(base + (size_t)kk * ld + H * D + h * D + dv);
        vreg[j] = *reinterpret_cast<const u32x4*>(base + (size_t)kk * ld + 2 * H * D + h * D + dv);
      }
    }
  };
  kv_load(0);
  for (int k0 = 0; k0 < L; k0 += KT) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int v = tid + j * 256;
      const int key = v / (D / VE), dv = (v % (D / VE)) * VE;
      *reinterpret_cast<u32x4*>(sK + key * KROW + dv * ES) = kreg[j];
      const T* ve = reinterpret_cast<const T*>(&vreg[j]);
#pragma unroll
      for (int e = 0; e < VE; ++e) *reinterpret_cast<T*>(sV + (dv + e) * VROW + key * ES) = ve[e];
    }
    __syncthreads();
    if (k0 + KT < L) kv_load(k0 + KT);

#pragma unroll
    for (int g = 0; g < QG; ++g) {
      // S^T tile: 4 m-subtiles of 16 keys x this wave's 16 queries.
      f32x4 s[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        s[mi] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < D / KSTEP; ++ks) {
          const int d0 = ks * KSTEP + lg * (KSTEP / 4);
          const u32x4 ka = *reinterpret_cast<const u32x4*>(sK + (mi * 16 + lr) * KROW + d0 * ES);
          Mma<T>::run(s[mi], ka, qf[g][ks]);
        }
      }
      // Online softmax over keys for this lane's query column, in the log2 domain: the running
      // max is kept pre-scaled by c = scale * log2(e), so each probability is one FMA and one
      // v_exp_f32: p = 2^(s * c - m) (c > 0, so the max of raw scores is the max of scaled).
      const float c = scale * 1.4426950408889634f;
      float tmax = -INFINITY;
      if (k0 + KT <= L) {                        // whole tile valid (every UNet shape)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[mi][r]);
      } else {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + mi * 16 + lg * 4 + r;
            if (key >= L) s[mi][r] = -INFINITY;
            tmax = fmaxf(tmax, s[mi][r]);
          }
      }
      tmax = red16_max(tmax);
      tmax = red32_max(tmax);
      const float mnew = fmaxf(mrun[g], tmax * c);
      const float corr = sizeof(T) == 2 ? __builtin_amdgcn_exp2f(mrun[g] - mnew) : exp2f(mrun[g] - mnew);
      float psum = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = fmaf(s[mi][r], c, -mnew);
          const float p = sizeof(T) == 2 ? __builtin_amdgcn_exp2f(a) : exp2f(a);
          s[mi][r] = p;
          psum += p;
        }
      psum = red16_sum(psum);
      psum = red32_sum(psum);
      lrun[g] = lrun[g] * corr + psum;
      mrun[g] = mnew;
#pragma unroll
      for (int i = 0; i < 2; ++i) oacc[g][i] *= corr;

      // O^T += V^T P^T over the 64 keys.
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {           // k-step = 32 keys = subtiles 2st, 2st+1
          typename Vec8<T>::t pb;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pb[j] = (T)s[2 * st][j];
            pb[4 + j] = (T)s[2 * st + 1][j];
          }
          const u32x4 pbu = __builtin_bit_cast(u32x4, pb);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const char* row = sV + (mi * 16 + lr) * VROW;
            uint2 lo = *reinterpret_cast<const uint2*>(row + (st * 32 + lg * 4) * ES);
            uint2 hi = *reinterpret_cast<const uint2*>(row + (st * 32 + 16 + lg * 4) * ES);
            Mma<T>::run(oacc[g][mi], u32x4{lo.x, lo.y, hi.x, hi.y}, pbu);
          }
        }
      } else {
#pragma unroll
        for (int st = 0; st < 4; ++st) {           // k-step = 16 keys = subtile st
          const u32x4 pbu = __builtin_bit_cast(u32x4, s[st]);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const u32x4 va = *reinterpret_cast<const u32x4*>(sV + (mi * 16 + lr) * VROW +
                                                             (st * 16 + lg * 4) * ES);
            Mma<T>::run(oacc[g][mi], va, pbu);
          }
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    if (qi[g] >= L) continue;
    const float inv = 1.f / lrun[g];
    T* out = o + ((size_t)b * L + qi[g]) * (H * D) + h * D;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[mi * 16 + lg * 4 + r] = from_f<T>(oacc[g][mi][r] * inv);
  }
}

// ------------------------------------------------------------------ K/V-resident variant
// flash_kv_kernel (bf16 / f16, L % 128 == 0, L <= 1024 — the UNet's 32x32 SpatialTransformer levels
// at 256^2): a block owns QG*128 queries of one (image, head) with 8 waves and keeps the head's
// WHOLE K and V in LDS (L x 64 B each, 128 KB at L = 1024):
//  * every K/V byte is DMA'd (global_load_lds, issued all at once in the prologue, 128-key
//    chunks in order) straight into LDS in its natural [key][d] layout, 16-byte chunk XOR-
//    swizzled by ((key >> 2) & 1) * 2 at the source (conflict-free for both reads below);
//    the only barriers are one per chunk as it lands, never a write-after-read;
//  * S^T = K Q^T: A = K rows (ds_read_b128), B = the wave's 16 queries (registers);
//  * O^T += V^T P^T: A = V^T read with ds_read_b64_tr_b16 (hardware transpose of the [key][d]
//    image), in exactly the key order the S^T accumulators hold P in (keys 4g..4g+3 and
//    16+4g..16+4g+3 of a 32-key step), so P feeds the MFMA straight from registers;
//  * each K / V fragment read serves all QG query groups of the wave; online softmax in the
//    log2 domain, the row sums kept per lane and reduced across lanes once at the end.
constexpr int FKV_NW = 8;
#ifndef DAC_FKV_SKIP
#define DAC_FKV_SKIP 1
#endif
DEV int fkv_swz(int key) { return ((key >> 2) & 1) << 1; }
template <int N> DEV void fkv_wait(int n) {
  // s_waitcnt vmcnt(n) for a runtime n in [0, N] (the immediate must be a constant).
  if constexpr (N > 0) {
    if (n >= N) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); return; }
    fkv_wait<N - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

//  * PRE (q prescaled by scale * log2(e), so scores come out in log2 units): the S^T MFMAs
//    start from C = -m (m the query's reference max) instead of 0, so p = 2^s' needs no
//    subtraction; m is only moved when some score of the wave passes it by more than 2^FKV_TAU
//    (p <= 2^8 fits T and the fp32 sums), the first chunk setting it. Exact: every p and every
//    rescale uses the same m, and the final 1/sum cancels it.
//  * JOINT (PRE): the wave's query groups walk a chunk together, in two 64-key halves,
//    so each K / V fragment read from LDS serves every group (the 16-wave form otherwise
//    re-reads them per group: half the LDS reads). m may move at either half (the first half of
//    the first chunk sets it): the same exact-in-m formulation at a finer step.
// The move test uses the lane's own max (any lane over TAU <=> some query's max over TAU); the
// cross-lane reduction to each query's max runs only on the rare move path.
constexpr float FKV_TAU = 8.f;
template <typename T, int QG, int NW = FKV_NW, bool PRE = false, bool JOINT = false>
__global__ void __launch_bounds__(64 * NW) flash_kv_kernel(const T* __restrict__ qkv, T* o, int L,
                                                          int H, float scale) {
  static_assert(NW == 8 || NW == 16, "8 waves (two per SIMD) or 16 (four per SIMD)");
  static_assert(!JOINT || PRE, "the joint group walk is built for the log2-domain form");
  constexpr int D = 32;
  extern __shared__ __attribute__((aligned(1024))) char fkv_smem[];
  char* sK = fkv_smem;
  char* sV = fkv_smem + (size_t)L * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xq = n / 8, xr = n % 8, xcd = id % 8;
  const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + id / 8;
  const int bx = t % gx, h = (t / gx) % gy, b = t / (gx * gy);
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;

  // Q fragments first (their loads retire before the K/V DMAs in vmcnt order).
  u32x4 qf[QG];
  int qi[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    qi[g] = bx * (NW * 16 * QG) + wave * (16 * QG) + g * 16 + lr;
    qf[g] = *reinterpret_cast<const u32x4*>(base + (size_t)qi[g] * ld + h * D + lg * 8);
  }
  // K / V DMA: instruction n fills keys 16n..16n+15 (1 KB); chunk c = instructions 8c..8c+7.
  // 8 waves: wave w issues instruction 8c + w of K and of V (2 per wave per chunk); 16 waves:
  // waves 0-7 issue K's, waves 8-15 V's (1 per wave per chunk).
  const int NC = L >> 7;
  constexpr int PER = NW == 8 ? 2 : 1;                // DMAs per wave per chunk
  {
    const int kl = lane >> 2, ch = lane & 3;
    for (int c = 0; c < NC; ++c) {
      const int nn = 8 * c + (wave & 7);
      const int key = 16 * nn + kl;
      const T* src = base + (size_t)key * ld + h * D + 8 * (ch ^ fkv_swz(key));
      if (NW == 8 || wave < 8)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + H * D),
                                         (__attribute__((address_space(3))) void*)(sK + nn * 1024), 16, 0, 0);
      if (NW == 8 || wave >= 8)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 2 * H * D),
                                         (__attribute__((address_space(3))) void*)(sV + nn * 1024), 16, 0, 0);
    }
  }

  // Row sums of P come out of the PV MFMAs: a third O^T tile whose A operand is all ones
  // (every row = sum over keys of P[q][key], in the same rounded P the numerator uses), so
  // no per-score add and no cross-lane reduction at the end.
  f32x4 oacc[QG][2], lacc[QG], mneg[QG];
  float mrun[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    oacc[g][0] = oacc[g][1] = lacc[g] = mneg[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    mrun[g] = PRE ? 0.f : -INFINITY;
  }
  const uint32_t one2 = std::is_same<T, f16>::value ? 0x3C003C00u : 0x3F803F80u;   // 1.0 in T, twice
  const u32x4 ones = u32x4{one2, one2, one2, one2};
  const float cs = scale * 1.4426950408889634f;
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

  int first = 1;                                 // opaque to the compiler: no peeled copy of chunk 0
  for (int c = 0; c < NC; ++c) {
    asm volatile("" : "+s"(first));
    fkv_wait<7 * PER>(PER * (NC - 1 - c));      // this wave's DMAs of chunk c have landed
    __builtin_amdgcn_s_barrier();                // ... and every other wave's
    asm volatile("" ::: "memory");
    const int kb = c * 128;
    auto kload = [&](int mi) -> u32x4 {
      const int key = kb + mi * 16 + lr;
      return *reinterpret_cast<const u32x4*>(sK + key * 64 + ((lg ^ fkv_swz(key)) << 4));
    };
    // V^T fragments: step st (32 keys), d tile dm: rows = keys, lane (4q+p) addresses key
    // kb + 32st + 4lg + q (+16), columns dm*16 + 4p .. +3.
    auto vload = [&](int st, int dm) -> u32x4 {
      uint32_t w[4];
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        const int key = kb + 32 * st + 16 * hi + 4 * lg + (lr >> 2);
        const int byte = (dm * 16 + 4 * (lr & 3)) * 2;          // 8-byte column group
        const int off = key * 64 + ((((byte >> 4) ^ fkv_swz(key)) << 4) | (byte & 15));
        const v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(sV + off));
        const uint2 u = __builtin_bit_cast(uint2, r);
        w[2 * hi] = u.x;
        w[2 * hi + 1] = u.y;
      }
      return u32x4{w[0], w[1], w[2], w[3]};
    };
    // 8 waves: the chunk's K / V fragments are read once and serve all QG groups; 16 waves
    // (128 VGPRs) re-read them per group instead of holding 64 registers of them.
    if constexpr (JOINT) {
      // Two 64-key halves (32 S^T registers per group live at a time, not 64).
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool fst = first && h == 0;
        f32x4 s[QG][4];
        u32x4 pbu[QG][2];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const u32x4 kf = kload(4 * h + mi);
#pragma unroll
          for (int g = 0; g < QG; ++g) {
            s[g][mi] = mneg[g];
            Mma<T>::run(s[g][mi], kf, qf[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          float lmax = s[g][0][0];
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) lmax = fmaxf(lmax, s[g][mi][r]);
          if (fst || __any(lmax > FKV_TAU)) {
            const float tmax = red32_max(red16_max(lmax));
            const float sh = fst ? tmax : fmaxf(tmax, 0.f);
            if (!fst) {
              const float corr = __builtin_amdgcn_exp2f(-sh);
              lacc[g] *= corr;
#pragma unroll
              for (int dm = 0; dm < 2; ++dm) oacc[g][dm] *= corr;
            }
            mrun[g] += sh;
            mneg[g] = f32x4{-mrun[g], -mrun[g], -mrun[g], -mrun[g]};
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
              s[g][mi] = mneg[g];
              Mma<T>::run(s[g][mi], kload(4 * h + mi), qf[g]);
            }
          }
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            typename Vec8<T>::t pb;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              pb[j] = (T)__builtin_amdgcn_exp2f(s[g][2 * s2][j]);
              pb[4 + j] = (T)__builtin_amdgcn_exp2f(s[g][2 * s2 + 1][j]);
            }
            pbu[g][s2] = __builtin_bit_cast(u32x4, pb);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int dm = 0; dm < 2; ++dm) {
            const u32x4 vf = vload(2 * h + s2, dm);
#pragma unroll
            for (int g = 0; g < QG; ++g) Mma<T>::run(oacc[g][dm], vf, pbu[g][s2]);
          }
#pragma unroll
          for (int g = 0; g < QG; ++g) Mma<T>::run(lacc[g], ones, pbu[g][s2]);
        }
      }
      first = 0;
      continue;
    }
    constexpr bool HOIST = NW == 8;
    u32x4 kf[HOIST ? 8 : 1], vf[HOIST ? 4 : 1][2];
    if constexpr (HOIST) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) kf[mi] = kload(mi);
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int dm = 0; dm < 2; ++dm) vf[st][dm] = vload(st, dm);
    }
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      if constexpr (!HOIST) asm volatile("" ::: "memory");
      f32x4 s[8];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        s[mi] = mneg[g];
        Mma<T>::run(s[mi], HOIST ? kf[mi] : kload(mi), qf[g]);
      }
      float tmax = s[0][0];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[mi][r]);
      if constexpr (PRE) {
        // s = score - m (log2 units). Rare case (the first chunk, or a score more than 2^TAU
        // above m): move m up to the chunk's max, rescale, and redo the S^T MFMAs from the new
        // -m, so both cases end in the same p = 2^s with no per-score subtraction.
        if (first || __any(tmax > FKV_TAU)) {
          tmax = red32_max(red16_max(tmax));
          const float sh = first ? tmax : fmaxf(tmax, 0.f);
          if (!first) {
            const float corr = __builtin_amdgcn_exp2f(-sh);
            lacc[g] *= corr;
#pragma unroll
            for (int dm = 0; dm < 2; ++dm) oacc[g][dm] *= corr;
          }
          mrun[g] += sh;
          mneg[g] = f32x4{-mrun[g], -mrun[g], -mrun[g], -mrun[g]};
          asm volatile("" ::: "memory");         // K re-read from LDS: kf need not stay live
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
            s[mi] = mneg[g];
            Mma<T>::run(s[mi], kload(mi), qf[g]);
          }
        }
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[mi][r] = __builtin_amdgcn_exp2f(s[mi][r]);
      } else {
        tmax = red32_max(red16_max(tmax));
        const float mnew = fmaxf(mrun[g], tmax * cs);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[mi][r] = __builtin_amdgcn_exp2f(fmaf(s[mi][r], cs, -mnew));
        // Rescale only when some query's running max moved (exact: otherwise corr == 1).
        if (DAC_FKV_SKIP == 0 || __any(mnew != mrun[g])) {
          const float corr = __builtin_amdgcn_exp2f(mrun[g] - mnew);
          lacc[g] *= corr;
#pragma unroll
          for (int dm = 0; dm < 2; ++dm) oacc[g][dm] *= corr;
        }
        mrun[g] = mnew;
      }
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        typename Vec8<T>::t pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (T)s[2 * st][j];
          pb[4 + j] = (T)s[2 * st + 1][j];
        }
        const u32x4 pbu = __builtin_bit_cast(u32x4, pb);
#pragma unroll
        for (int dm = 0; dm < 2; ++dm) Mma<T>::run(oacc[g][dm], HOIST ? vf[st][dm] : vload(st, dm), pbu);
        Mma<T>::run(lacc[g], ones, pbu);
      }
    }
    first = 0;
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const float inv = 1.f / lacc[g][0];          // every row of the ones tile holds query lr's sum
    T* out = o + ((size_t)b * L + qi[g]) * (H * D) + h * D;
#pragma unroll
    for (int dm = 0; dm < 2; ++dm) {
      typename Vec8<T>::t2 v0, v1;
      v0[0] = (T)(oacc[g][dm][0] * inv); v0[1] = (T)(oacc[g][dm][1] * inv);
      v1[0] = (T)(oacc[g][dm][2] * inv); v1[1] = (T)(oacc[g][dm][3] * inv);
      uint2 st;
      st.x = __builtin_bit_cast(uint32_t, v0);
      st.y = __builtin_bit_cast(uint32_t, v1);
      *reinterpret_cast<uint2*>(out + dm * 16 + 4 * lg) = st;
    }
  }
}

// ------------------------------------------------------------------ K/V-ring variant
// flash_kr_kernel (bf16 / f16, L % 64 == 0): the same transposed MFMA formulation and LDS image
// as flash_kv, but K / V stream through a 3-slot ring of 64-key chunks (8 KB a slot, 24 KB a
// block) instead of being resident (128 KB), and a block is 4 waves x QG x 16 queries. Four
// blocks then share a CU (16 waves, against flash_kv's 8), so one wave's S -> max -> exp -> PV
// chain overlaps other waves' MFMAs. Each chunk is one barrier: at chunk c the slot of chunk c-1
// (read by every wave before that barrier) is refilled with chunk c+2.
constexpr int FKR_NW = 4, FKR_NST = 3, FKR_CK = 64;
template <typename T, int QG>
__global__ void __launch_bounds__(64 * FKR_NW) flash_kr_kernel(const T* __restrict__ qkv, T* o, int L,
                                                              int H, float scale) {
  constexpr int D = 32, SLOT = FKR_CK * 64;          // bytes of one K (or V) chunk
  __shared__ __attribute__((aligned(1024))) char smem[2 * FKR_NST * SLOT];
  char* sK = smem;
  char* sV = smem + FKR_NST * SLOT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xq = n / 8, xr = n % 8, xcd = id % 8;
  const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + id / 8;
  const int bx = t % gx, h = (t / gx) % gy, b = t / (gx * gy);
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;

  u32x4 qf[QG];
  int qi[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    qi[g] = bx * (FKR_NW * 16 * QG) + wave * (16 * QG) + g * 16 + lr;
    qf[g] = *reinterpret_cast<const u32x4*>(base + (size_t)qi[g] * ld + h * D + lg * 8);
  }
  // Chunk c -> slot c % NST: wave w fills keys 16w .. 16w+15 of the chunk, of K and of V.
  const int NC = L / FKR_CK;
  auto issue = [&](int c) {
    const int kl = 16 * wave + (lane >> 2), ch = lane & 3;
    const T* src = base + (size_t)(c * FKR_CK + kl) * ld + h * D + 8 * (ch ^ fkv_swz(kl));
    char* dk = sK + (c % FKR_NST) * SLOT + wave * 1024;
    char* dv = sV + (c % FKR_NST) * SLOT + wave * 1024;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + H * D),
                                     (__attribute__((address_space(3))) void*)dk, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 2 * H * D),
                                     (__attribute__((address_space(3))) void*)dv, 16, 0, 0);
  };
#pragma unroll
  for (int c = 0; c < FKR_NST - 1; ++c)
    if (c < NC) issue(c);

  f32x4 oacc[QG][2], lacc[QG];
  float mrun[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    oacc[g][0] = oacc[g][1] = lacc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    mrun[g] = -INFINITY;
  }
  const uint32_t one2 = std::is_same<T, f16>::value ? 0x3C003C00u : 0x3F803F80u;
  const u32x4 ones = u32x4{one2, one2, one2, one2};
  const float cs = scale * 1.4426950408889634f;
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

  for (int c = 0; c < NC; ++c) {
    // This wave's DMAs of chunk c landed (the chunks issued after it may stay in flight), then
    // every wave's; after the barrier no wave still reads chunk c-1's slot.
    const int younger = NC - 1 - c < FKR_NST - 2 ? NC - 1 - c : FKR_NST - 2;
    fkv_wait<2 * (FKR_NST - 2)>(2 * younger);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + FKR_NST - 1 < NC) issue(c + FKR_NST - 1);
    const char* k0 = sK + (c % FKR_NST) * SLOT;
    const char* v0 = sV + (c % FKR_NST) * SLOT;
    u32x4 kf[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int key = mi * 16 + lr;
      kf[mi] = *reinterpret_cast<const u32x4*>(k0 + key * 64 + ((lg ^ fkv_swz(key)) << 4));
    }
    u32x4 vf[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int dm = 0; dm < 2; ++dm) {
        uint32_t w[4];
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
          const int key = 32 * st + 16 * hi + 4 * lg + (lr >> 2);
          const int byte = (dm * 16 + 4 * (lr & 3)) * 2;
          const int off = key * 64 + ((((byte >> 4) ^ fkv_swz(key)) << 4) | (byte & 15));
          const v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(v0 + off));
          const uint2 u = __builtin_bit_cast(uint2, r);
          w[2 * hi] = u.x;
          w[2 * hi + 1] = u.y;
        }
        vf[st][dm] = u32x4{w[0], w[1], w[2], w[3]};
      }
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      f32x4 s[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        s[mi] = f32x4{0.f, 0.f, 0.f, 0.f};
        Mma<T>::run(s[mi], kf[mi], qf[g]);
      }
      float tmax = s[0][0];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[mi][r]);
      tmax = red16_max(tmax);
      tmax = red32_max(tmax);
      const float mnew = fmaxf(mrun[g], tmax * cs);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[mi][r] = __builtin_amdgcn_exp2f(fmaf(s[mi][r], cs, -mnew));
      if (DAC_FKV_SKIP == 0 || __any(mnew != mrun[g])) {
        const float corr = __builtin_amdgcn_exp2f(mrun[g] - mnew);
        lacc[g] *= corr;
#pragma unroll
        for (int dm = 0; dm < 2; ++dm) oacc[g][dm] *= corr;
      }
      mrun[g] = mnew;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        typename Vec8<T>::t pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (T)s[2 * st][j];
          pb[4 + j] = (T)s[2 * st + 1][j];
        }
        const u32x4 pbu = __builtin_bit_cast(u32x4, pb);
#pragma unroll
        for (int dm = 0; dm < 2; ++dm) Mma<T>::run(oacc[g][dm], vf[st][dm], pbu);
        Mma<T>::run(lacc[g], ones, pbu);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const float inv = 1.f / lacc[g][0];
    T* out = o + ((size_t)b * L + qi[g]) * (H * D) + h * D;
#pragma unroll
    for (int dm = 0; dm < 2; ++dm) {
      typename Vec8<T>::t2 v0, v1;
      v0[0] = (T)(oacc[g][dm][0] * inv); v0[1] = (T)(oacc[g][dm][1] * inv);
      v1[0] = (T)(oacc[g][dm][2] * inv); v1[1] = (T)(oacc[g][dm][3] * inv);
      uint2 stv;
      stv.x = __builtin_bit_cast(uint32_t, v0);
      stv.y = __builtin_bit_cast(uint32_t, v1);
      *reinterpret_cast<uint2*>(out + dm * 16 + 4 * lg) = stv;
    }
  }
}
// 1: the K/V-ring kernel is the dispatcher's choice for the L <= 1024 shapes (DAC_FLASH_KR).
int g_flash_kr = getenv("DAC_FLASH_KR") ? atoi(getenv("DAC_FLASH_KR")) : 0;

// 1: the 16-wave flash_kv (four waves per SIMD, two query groups each) is the dispatcher's
// choice for the K/V-resident shapes (DAC_FKV16).
int g_fkv16 = getenv("DAC_FKV16") ? atoi(getenv("DAC_FKV16")) : 0;

// 1 (default): the 16-wave log2-domain kernel walks its two query groups jointly (DAC_FKV_JOINT;
// 28.0 -> 26.6 us at C = 512, B = 8 standalone, tools/attn_bench.py).
int g_fkv_joint = getenv("DAC_FKV_JOINT") ? atoi(getenv("DAC_FKV_JOINT")) : 1;

template <typename T, int QG, int NW, bool PRE, bool JOINT = false>
static void fkv_launch(const void* qkv, void* o, int B, int L, int H, float scale, hipStream_t st) {
  // > 64 KB of dynamic LDS must be opted into, once per (kernel, device).
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev >= 64) dev = 63;
  const uint64_t bit = 1ull << dev;
  if (!(done.load(std::memory_order_acquire) & bit)) {
    (void)hipFuncSetAttribute((const void*)flash_kv_kernel<T, QG, NW, PRE, JOINT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              131072);
    done.fetch_or(bit, std::memory_order_acq_rel);
  }
  const dim3 g(L / (NW * 16 * QG), H, B);
  flash_kv_kernel<T, QG, NW, PRE, JOINT><<<g, 64 * NW, (size_t)L * 128, st>>>((const T*)qkv, (T*)o, L, H, scale);
}

// variant: 0 = the dispatcher's choice (g_flash_old = DAC_FLASH_OLD selects the staged-tile
// kernel process-wide, g_flash_kr = DAC_FLASH_KR the K/V-ring one), 1 = the staged-tile kernel,
// 2 = the K/V-ring kernel (16-bit, L % 64 == 0), 3 = the 16-wave K/V-resident kernel (16-bit,
// L % 256 == 0, L <= 1024), 4 = its two-group joint walk (16-bit, prescaled q, L % 512 == 0,
// L <= 1024; else as 3). Passed explicitly by the op-level test hook, so no global state is
// toggled per call. scale == 0: q was prescaled by 32^-0.5 * log2(e) (the engine's 16-bit
// q|k|v weights), scores are already in log2 units.
template <typename T>
void flash_attn_d32_v(const void* qkv, void* o, int B, int L, int H, float scale, int variant, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    const bool pre = scale == 0.f;
    const bool kv = L % 128 == 0 && L <= 1024 && variant == 0 && !g_flash_old && !g_flash_kr;
    if (variant == 4 && pre && L % 512 == 0 && L <= 1024) {
      fkv_launch<T, 2, 16, true, true>(qkv, o, B, L, H, scale, st);
      return;
    }
    if (L % 256 == 0 && L <= 1024 && (variant == 3 || variant == 4 || (kv && (pre || g_fkv16)))) {
      // 16 waves x 2 query groups: the same 512 queries per block as the 8-wave QG = 4 kernel,
      // with four waves per SIMD to overlap one wave's S -> max -> exp -> PV chain; one query
      // group per wave (256 queries per block) when 512 would leave CUs idle. The log2-domain
      // (prescaled q) kernels are built only in this form and the QG = 1 8-wave one (the
      // 8-wave QG = 4 form spills with the extra -m operands).
      const bool two = L % 512 == 0 && (long)(L / 512) * H * B >= 256;
      if (pre) {
        // One query group per wave takes the same walk (64-key halves) as the joint two-group
        // kernel: the per-group arithmetic -- and so every output -- is then the same whichever
        // of the two the batch size selects (batch- and shard-invariance).
        if (two && g_fkv_joint) fkv_launch<T, 2, 16, true, true>(qkv, o, B, L, H, scale, st);
        else if (two) fkv_launch<T, 2, 16, true>(qkv, o, B, L, H, scale, st);
        else if (g_fkv_joint) fkv_launch<T, 1, 16, true, true>(qkv, o, B, L, H, scale, st);
        else fkv_launch<T, 1, 16, true>(qkv, o, B, L, H, scale, st);
      } else {
        if (two) fkv_launch<T, 2, 16, false>(qkv, o, B, L, H, scale, st);
        else fkv_launch<T, 1, 16, false>(qkv, o, B, L, H, scale, st);
      }
      return;
    }
    if (kv) {
      // K/V-resident kernel: 4 query groups per wave (512 queries per block) when that still
      // fills the chip, else 2 (or 1).
      if (pre && g_fkv_joint) fkv_launch<T, 1, FKV_NW, true, true>(qkv, o, B, L, H, scale, st);
      else if (pre) fkv_launch<T, 1, FKV_NW, true>(qkv, o, B, L, H, scale, st);
      else if (L % 512 == 0 && (long)(L / 512) * H * B >= 256) fkv_launch<T, 4, FKV_NW, false>(qkv, o, B, L, H, scale, st);
      else if (L % 256 == 0) fkv_launch<T, 2, FKV_NW, false>(qkv, o, B, L, H, scale, st);
      else fkv_launch<T, 1, FKV_NW, false>(qkv, o, B, L, H, scale, st);
      return;
    }
  }
  // The other kernels take the multiplier: prescaled scores need 1 / log2(e).
  if (scale == 0.f) scale = 0.6931471805599453f;
  if constexpr (sizeof(T) == 2) {
    if (L % 64 == 0 && (variant == 2 || (variant == 0 && g_flash_kr && !g_flash_old && L % 128 == 0 && L <= 1024))) {
      // K/V-ring kernel: 2 query groups per wave (128 queries per block) while that leaves
      // >= 1024 blocks (4 per CU), else 1.
      if (L % 128 == 0 && (long)(L / 128) * H * B >= 1024) {
        dim3 g(L / 128, H, B);
        flash_kr_kernel<T, 2><<<g, 64 * FKR_NW, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
      } else {
        dim3 g(L / 64, H, B);
        flash_kr_kernel<T, 1><<<g, 64 * FKR_NW, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
      }
      return;
    }
  }
  // Two 16-query groups per wave (128 queries per block) once that still leaves >= 2 blocks
  // per CU: each staged K/V tile and its two barriers then serve twice the queries.
  if ((long)((L + 127) / 128) * H * B >= 512) {
    dim3 g((L + 127) / 128, H, B);
    flash_d32_kernel<T, 2><<<g, 256, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
  } else {
    dim3 g((L + 63) / 64, H, B);
    flash_d32_kernel<T, 1><<<g, 256, 0, st>>>((const T*)qkv, (T*)o, L, H, scale);
  }
}

// ------------------------------------------------------------------------------ small MHA
// Short-sequence MHA (ViT tokens L = 50 / 257, CLIP text L = 77), head dim 64 (or 32): four
// threads per query, each owning D/4 of the head dimensions (partial q.k dot products summed
// over the quad with DPP), K / V of the (image, head) staged in LDS as fp32, single-pass online
// softmax (running max + rescaled accumulator, so any L fits in registers); `causal` masks keys
// t > query (the text tower's additive -inf upper triangle, transformer.py:751-757).
template <int CTRL> DEV float dpp_quad(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <typename T, int D>
__global__ void __launch_bounds__(256) small_mha_kernel(const T* __restrict__ qkv, T* o, int L, int H,
                                                        int causal) {
  constexpr int DP = D / 4;                   // dims per thread
  extern __shared__ float sm[];               // K [L][D], V [L][D]
  const int b = blockIdx.y, h = blockIdx.x;
  const int ld = 3 * H * D;
  const T* base = qkv + (size_t)b * L * ld;
  float* sk = sm;
  float* sv = sm + L * D;
  for (int i = threadIdx.x; i < L * D; i += 256) {
    const int t = i / D, d = i - t * D;
    sk[i] = to_f(base[(size_t)t * ld + H * D + h * D + d]);
    sv[i] = to_f(base[(size_t)t * ld + 2 * H * D + h * D + d]);
  }
  __syncthreads();
  const float scale = rsqrtf((float)D);
  const int part = threadIdx.x & 3, d0 = part * DP;
  for (int qi = blockIdx.z * 64 + (threadIdx.x >> 2); qi < L; qi += 64 * gridDim.z) {
    // (the quad's four lanes share qi, so the loop bound and the causal limit are quad-uniform)
    float qv[DP], acc[DP];
#pragma unroll
    for (int d = 0; d < DP; ++d) { qv[d] = to_f(base[(size_t)qi * ld + h * D + d0 + d]) * scale; acc[d] = 0.f; }
    float mx = -INFINITY, sum = 0.f;
    const int tend = causal ? qi + 1 : L;
    for (int t = 0; t < tend; ++t) {
      const float* kr = sk + t * D + d0;
      float a = 0.f;
#pragma unroll
      for (int d = 0; d < DP; ++d) a += qv[d] * kr[d];
      a += dpp_quad<0xB1>(a);                 // quad_perm [1,0,3,2]
      a += dpp_quad<0x4E>(a);                 // quad_perm [2,3,0,1]
      const float mn = fmaxf(mx, a);
      const float c = expf(mx - mn), p = expf(a - mn);
      sum = sum * c + p;
      const float* vr = sv + t * D + d0;
#pragma unroll
      for (int d = 0; d < DP; ++d) acc[d] = acc[d] * c + p * vr[d];
      mx = mn;
    }
    const float inv = 1.f / sum;
    T* out = o + ((size_t)b * L + qi) * (H * D) + h * D + d0;
#pragma unroll
    for (int d = 0; d < DP; ++d) out[d] = from_f<T>(acc[d] * inv);
  }
}

template <typename T>
void small_mha(const void* qkv, void* o, int B, int L, int H, int D, int causal, hipStream_t st) {
  const size_t smem = (size_t)L * 2 * D * sizeof(float);
  const dim3 g(H, B, (L + 63) / 64);
  if (D == 64) small_mha_kernel<T, 64><<<g, 256, smem, st>>>((const T*)qkv, (T*)o, L, H, causal);
  else if (D == 32) small_mha_kernel<T, 32><<<g, 256, smem, st>>>((const T*)qkv, (T*)o, L, H, causal);
  else throw std::invalid_argument("small_mha: head dim must be 32 or 64");
}

template <typename T>
void flash_attn_d32(const void* qkv, void* o, int B, int L, int H, float scale, hipStream_t st) {
  flash_attn_d32_v<T>(qkv, o, B, L, H, scale, 0, st);
}

#define INST(T)                                                                           \
  template void flash_attn_d32<T>(const void*, void*, int, int, int, float, hipStream_t); \
  template void flash_attn_d32_v<T>(const void*, void*, int, int, int, float, int, hipStream_t); \
  template void small_mha<T>(const void*, void*, int, int, int, int, int, hipStream_t);
INST(float)
INST(bf16)
INST(f16)
#undef INST

}  // namespace dac
