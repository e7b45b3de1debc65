// misc.hip — small kernels around the two networks:
//  * small_linear / softmax_mul : fp32 per-image MLPs (time_mlp, text_mlp, prompt_mlp,
//    ResBlock.mlp, cross-attention value path, ViT head), DenoisingUNet_arch.py:51-63,
//    132-137; module_util.py:135-137, 143-148; transformer.py:546-547.
//  * unet_prep / unet_out : input concat + reflect pad, output crop (DenoisingUNet_arch.py:
//    123-127, 172).
//  * sde_step : IR-SDE posterior / reverse-SDE update with injected or Philox noise
//    (sde_utils.py:44-45, 177-187, 205-231, 245-247).
//  * vit_prep / vit_embed / rows_to_f32 : ViT stem and pooled-token extraction
//    (transformer.py:518-532, 543-544).
#include "common.h"
#include "kernels.h"

#include <cmath>
#include <cstdlib>

namespace dac {

__device__ __forceinline__ float act_f(float v, int a) {
  return a == ACT_SILU ? silu_f(v) : a == ACT_GELU ? gelu_f(v) : v;
}

// Block = SL_R rows x 32 outputs, one thread per (row, output): the block's input rows are
// staged in LDS once (with the pre-activation) and every W row is read by the SL_R threads of
// its output from L1/L2 (16-byte loads), instead of once per (row, 32 outputs) block; each
// output is one thread's fixed-order sum, so results do not depend on R (batch invariance).
constexpr int SL_R = 8;
__global__ void __launch_bounds__(256) small_linear_kernel(const float* __restrict__ x, int ldx,
                                                           const float* __restrict__ W,
                                                           const float* b, float* y, int ldy,
                                                           int R, int I, int O, int pre,
                                                           int post, const float* add,
                                                           int add_ld, int add_mod) {
  extern __shared__ float xs[];                 // [SL_R][I]
  const int r0 = blockIdx.y * SL_R;
  for (int k = threadIdx.x; k < SL_R * I; k += 256) {
    const int rr = k / I, i = k - rr * I;
    xs[k] = r0 + rr < R ? act_f(x[(size_t)(r0 + rr) * ldx + i], pre) : 0.f;
  }
  __syncthreads();
  const int rr = threadIdx.x >> 5, o = blockIdx.x * 32 + (threadIdx.x & 31), r = r0 + rr;
  if (o >= O || r >= R) return;
  const float* wr = W + (size_t)o * I;
  const float* xr = xs + rr * I;
  float s = 0.f;
  if ((I & 3) == 0 && ((uintptr_t)W & 15) == 0) {
    // Four independent partial sums (combined in a fixed order): the FMA chain is not one
    // I-long dependency.
    float s4[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < I; i += 4) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(wr + i);
      const f32x4 xv = *reinterpret_cast<const f32x4*>(xr + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) s4[e] = fmaf(xv[e], w[e], s4[e]);
    }
    s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  } else {
    for (int i = 0; i < I; ++i) s = fmaf(xr[i], wr[i], s);
  }
  float v = s + (b ? b[o] : 0.f);
  v = act_f(v, post);
  if (add) v += add[(size_t)(r % add_mod) * add_ld + o];
  y[(size_t)r * ldy + o] = v;
}

void small_linear(const float* x, int ldx, const float* W, const float* b, float* y, int ldy,
                  int R, int I, int O, int pre, int post, const float* add, int add_ld,
                  int add_mod, hipStream_t st) {
  dim3 g((O + 31) / 32, (R + SL_R - 1) / SL_R);
  small_linear_kernel<<<g, 256, SL_R * I * sizeof(float), st>>>(x, ldx, W, b, y, ldy, R, I, O, pre,
                                                                 post, add, add_ld, add_mod > 0 ? add_mod : 1);
}

__global__ void __launch_bounds__(256) softmax_mul_kernel(const float* x, const float* v,
                                                          float* y, int C) {
  const int r = blockIdx.x;
  __shared__ float red[4];
  __shared__ float bc;
  const float* xr = x + (size_t)r * C;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < C; i += 256) m = fmaxf(m, xr[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) bc = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  m = bc;
  float s = 0.f;
  for (int i = threadIdx.x; i < C; i += 256) s += expf(xr[i] - m);
  s = wave_sum(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bc = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += 256) y[(size_t)r * C + i] = expf(xr[i] - m) / bc * v[i];
}

void softmax_mul(const float* x, const float* v, float* y, int R, int C, hipStream_t st) {
  softmax_mul_kernel<<<R, 256, 0, st>>>(x, v, y, C);
}

// SinusoidalPosEmb (module_util.py:41-48) for R = n_t * B rows: row r uses the time
// t = float((t0 + dt * (r / B)) * scale), i.e. the reference's python `t * self.sample_scale`
// (sde_utils.py:197, 202, 302; a double) rounded once to the float32 time tensor
// (DenoisingUNet_arch.py:120-121); emb = exp(k * -(ln(10000) / (half - 1))) in fp32.
__global__ void sinus_kernel(float* out, int R, int B, int nf, double t0, double dt, double scale,
                             float negemb) {
  const int half = nf / 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= R * half) return;
  const int r = i / half, k = i - r * half;
  const float t = (float)((t0 + dt * (double)(r / B)) * scale);
  const float a = t * expf((float)k * negemb);
  out[(size_t)r * nf + k] = sinf(a);
  out[(size_t)r * nf + half + k] = cosf(a);
}

void sinus_embedding(float* out, int R, int B, int nf, double t0, double dt, double scale,
                     hipStream_t st) {
  const int half = nf / 2;
  const float negemb = (float)(-(std::log(10000.0) / (half - 1)));
  sinus_kernel<<<(R * half + 255) / 256, 256, 0, st>>>(out, R, B, nf, t0, dt, scale, negemb);
}

// Precision analysis (DAC_EMU_A, engine.cpp): round fp32 rows to bf16 in place, as a bf16
// store followed by a load would (round to nearest even).
// fp16 != 0 rounds to IEEE half instead (DAC_EMU_FP16: what fp16 storage would cost).
__global__ void round_bf16_kernel(float* y, int ld, size_t rows, int C, int fp16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * C) return;
  float* p = y + (i / C) * ld + i % C;
  *p = fp16 ? (float)(_Float16)(*p) : (float)(bf16)(*p);
}
void round_bf16_rows(float* y, int ld, size_t rows, int C, hipStream_t st) {
  const size_t n = rows * C;
  static const int h = getenv("DAC_EMU_FP16") ? atoi(getenv("DAC_EMU_FP16")) : 0;
  if (n) round_bf16_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(y, ld, rows, C, h);
}

__global__ void ss_fill_kernel(float* ss, int C, float scale_m1, const float* shift) {
  for (int c = threadIdx.x; c < C; c += 256) {
    ss[c] = scale_m1;
    ss[C + c] = shift ? shift[c] : 0.f;
  }
}
void ss_fill(float* ss, int C, float scale_m1, const float* shift, hipStream_t st) {
  ss_fill_kernel<<<1, 256, 0, st>>>(ss, C, scale_m1, shift);
}

// Stage the loop's noise key on the device in stream order (kernel arguments, no host
// staging buffer and no host synchronisation).
__global__ void set_u64x2_kernel(uint64_t* p, uint64_t a, uint64_t b) {
  if (threadIdx.x == 0) { p[0] = a; p[1] = b; }
}
__global__ void stamp_init_kernel(unsigned long long* s, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) { s[2 * i] = ~0ull; s[2 * i + 1] = 0ull; }
}
void stamp_init(unsigned long long* s, size_t n, hipStream_t st) {
  if (n) stamp_init_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(s, n);
}
void set_u64x2(uint64_t* p, uint64_t a, uint64_t b, hipStream_t st) {
  set_u64x2_kernel<<<1, 64, 0, st>>>(p, a, b);
}

// --------------------------------------------------------------------------- UNet I/O
template <typename T>
__global__ void unet_prep_kernel(const float* xt, const float* mu, T* x, int B, int H, int W,
                                 int Hp, int Wp) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t n = (size_t)B * Hp * Wp;
  if (i >= n) return;
  const int w = (int)(i % Wp);
  const int h = (int)((i / Wp) % Hp);
  const int b = (int)(i / ((size_t)Wp * Hp));
  const int sh = h < H ? h : 2 * (H - 1) - h;     // F.pad(..., 'reflect')
  const int sw = w < W ? w : 2 * (W - 1) - w;
  float v[8];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const size_t o = (((size_t)b * 3 + c) * H + sh) * W + sw;
    const float m = mu[o];
    v[c] = xt[o] - m;
    v[3 + c] = m;
  }
  v[6] = v[7] = 0.f;
  T* dst = x + i * 8;
  if constexpr (sizeof(T) == 2) {
    store_vec<T>(dst, v);
  } else {
    store_vec<T>(dst, v);
    store_vec<T>(dst + 4, v + 4);
  }
}

template <typename T>
void unet_prep(const float* xt, const float* mu, void* x, int B, int H, int W, int Hp, int Wp,
               hipStream_t st) {
  const size_t n = (size_t)B * Hp * Wp;
  unet_prep_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(xt, mu, (T*)x, B, H, W, Hp, Wp);
}

template <typename T>
__global__ void unet_out_kernel(const T* y, int ld, float* eps, int B, int H, int W, int Hp,
                                int Wp) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t n = (size_t)B * 3 * H * W;
  if (i >= n) return;
  const int w = (int)(i % W);
  const int h = (int)((i / W) % H);
  const int c = (int)((i / ((size_t)W * H)) % 3);
  const int b = (int)(i / ((size_t)W * H * 3));
  eps[i] = to_f(y[(((size_t)b * Hp + h) * Wp + w) * ld + c]);
}

template <typename T>
void unet_out(const void* y, int ld, float* eps, int B, int H, int W, int Hp, int Wp,
              hipStream_t st) {
  const size_t n = (size_t)B * 3 * H * W;
  unet_out_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const T*)y, ld, eps, B, H, W,
                                                                  Hp, Wp);
}

// --------------------------------------------------------------------------- sampler
// Philox4x32-10 counter-based generator (Salmon et al., SC'11), Box-Muller to N(0,1).
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float philox_normal(uint64_t seed, uint32_t tag, uint64_t i) {
  const uint4 r = philox(make_uint4((uint32_t)(i >> 1), (uint32_t)(i >> 33), tag, 0x5DAC11Fu),
                         make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float u1 = ((i & 1 ? r.z : r.x) >> 8) * (1.f / 16777216.f) + (0.5f / 16777216.f);
  const float u2 = ((i & 1 ? r.w : r.y) >> 8) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}

template <typename T>
__global__ void sde_step_kernel(int mode, float* x, const float* mu, const T* eps, int ld, int Hp,
                                int Wp, const float* z, const uint64_t* seedp, uint32_t tag,
                                StepCoef c, int H, int W, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int w = (int)(i % W);
  const int h = (int)((i / W) % H);
  const int ch = (int)((i / ((size_t)W * H)) % 3);
  const int b = (int)(i / ((size_t)W * H * 3));
  const float e = ld == 0 ? to_f(eps[i]) : to_f(eps[(((size_t)b * Hp + h) * Wp + w) * ld + ch]);
  const float xv = x[i], m = mu[i];
  const float zv = z ? z[i] : philox_normal(seedp[0], tag, i + seedp[1]);
  float out;
  if (mode == 0) {
    const float x0 = ((xv - m) - c.sbar * e) * c.ea + m;                  // sde_utils.py:245-247
    const float mean = c.t1 * (xv - m) + c.t2 * (x0 - m) + m;             // :205-213
    out = mean + c.std * zv;                                              // :227-231
  } else {
    const float score = -e / c.sbar;                                      // :186-187
    const float drift = (c.theta * (m - xv) - c.sigma2 * score) * c.dt;   // :177-178
    out = xv - drift - c.sigma_sqrt_dt * zv;                              // :44-45, 183-184
  }
  x[i] = out;
}

// The loop form (eps = the final conv's NHWC output, ld channels a pixel): one thread per pixel
// and all three channels, so eps is read as one contiguous run per pixel instead of three
// scattered 2-byte reads from three planes' threads. Same per-element arithmetic, noise key and
// output as sde_step_kernel (bit-identical).
template <typename T>
__global__ void sde_step_px_kernel(int mode, float* x, const float* mu, const T* eps, int ld, int Hp,
                                   int Wp, const float* z, const uint64_t* seedp, uint32_t tag,
                                   StepCoef c, int H, int W, size_t npx, T* xin) {
  const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= npx) return;
  const int w = (int)(p % W);
  const int h = (int)((p / W) % H);
  const int b = (int)(p / ((size_t)W * H));
  const T* ep = eps + (((size_t)b * Hp + h) * Wp + w) * ld;
  float e3[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) e3[ch] = to_f(ep[ch]);
  const size_t plane = (size_t)H * W;
  float v[8];                                   // next step's input row (unet_prep_kernel's)
  v[6] = v[7] = 0.f;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const size_t i = ((size_t)b * 3 + ch) * plane + (size_t)h * W + w;
    const float e = e3[ch];
    const float xv = x[i], m = mu[i];
    const float zv = z ? z[i] : philox_normal(seedp[0], tag, i + seedp[1]);
    float out;
    if (mode == 0) {
      const float x0 = ((xv - m) - c.sbar * e) * c.ea + m;                  // sde_utils.py:245-247
      const float mean = c.t1 * (xv - m) + c.t2 * (x0 - m) + m;             // :205-213
      out = mean + c.std * zv;                                              // :227-231
    } else {
      const float score = -e / c.sbar;                                      // :186-187
      const float drift = (c.theta * (m - xv) - c.sigma2 * score) * c.dt;   // :177-178
      out = xv - drift - c.sigma_sqrt_dt * zv;                              // :44-45, 183-184
    }
    x[i] = out;
    v[ch] = out - m;
    v[3 + ch] = m;
  }
  if (xin) {                                    // (Hp == H, Wp == W: pixel p is input row p)
    T* dst = xin + p * 8;
    store_vec<T>(dst, v);
    if constexpr (sizeof(T) == 4) store_vec<T>(dst + 4, v + 4);
  }
}

static bool sde_px_on() {                       // read per call: tests toggle it per handle
  return !(getenv("DAC_SDE_PX") && atoi(getenv("DAC_SDE_PX")) == 0);
}
bool sde_step_fuses(int ld, int H, int W, int Hp, int Wp) { return sde_px_on() && ld >= 3 && Hp == H && Wp == W; }

template <typename T>
void sde_step(int mode, float* x, const float* mu, const void* eps, int ld, int Hp, int Wp,
              const float* z, const uint64_t* seedp, uint32_t tag, StepCoef c, int B, int H,
              int W, hipStream_t st, void* xin) {
  if (xin && !sde_step_fuses(ld, H, W, Hp, Wp)) throw std::invalid_argument("sde_step: fused input write needs the per-pixel kernel on unpadded images");
  if (ld >= 3 && sde_px_on()) {
    const size_t npx = (size_t)B * H * W;
    sde_step_px_kernel<T><<<(unsigned)((npx + 255) / 256), 256, 0, st>>>(mode, x, mu, (const T*)eps, ld, Hp, Wp,
                                                                         z, seedp, tag, c, H, W, npx, (T*)xin);
    return;
  }
  const size_t n = (size_t)B * 3 * H * W;
  sde_step_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(mode, x, mu, (const T*)eps, ld,
                                                                  Hp, Wp, z, seedp, tag, c, H, W, n);
}

// --------------------------------------------------------------------------- ViT stem
template <typename T>
__global__ void vit_prep_kernel(const float* img, T* x, int B, int S) {
  constexpr int VE = TypeInfo<T>::VE;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t n = (size_t)B * S * S;
  if (i >= n) return;
  const int w = (int)(i % S), h = (int)((i / S) % S), b = (int)(i / ((size_t)S * S));
  float v[VE];
#pragma unroll
  for (int c = 0; c < VE; ++c) v[c] = c < 3 ? img[(((size_t)b * 3 + c) * S + h) * S + w] : 0.f;
  store_vec<T>(x + i * VE, v);
}

template <typename T>
void vit_prep(const float* img, void* x, int B, int S, hipStream_t st) {
  const size_t n = (size_t)B * S * S;
  vit_prep_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(img, (T*)x, B, S);
}

// ViT stem as a GEMM: the patch conv has stride == kernel, so im2col is a pure gather.
// x[(b * G*G + py * G + px) * K + (ky * P + kx) * 3 + c] = img[b][c][py P + ky][px P + kx],
// K = 3 P P (the packed weight order [D][ky][kx][3]).
template <typename T>
__global__ void vit_patches_kernel(const float* img, T* x, int S, int P, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int K = 3 * P * P, G = S / P;
  const int k = (int)(i % K);
  const size_t row = i / K;
  const int p = (int)(row % ((size_t)G * G));
  const int b = (int)(row / ((size_t)G * G));
  const int c = k % 3, kx = (k / 3) % P, ky = k / (3 * P);
  const int py = p / G, px = p - py * G;
  x[i] = from_f<T>(img[(((size_t)b * 3 + c) * S + py * P + ky) * S + px * P + kx]);
}

template <typename T>
void vit_patches(const float* img, void* x, int B, int S, int P, hipStream_t st) {
  const size_t n = (size_t)B * (S / P) * (S / P) * 3 * P * P;
  vit_patches_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(img, (T*)x, S, P, n);
}

template <typename T>
__global__ void vit_embed_kernel(const T* patch, const float* cls, const float* pos, T* tok,
                                 int L, int D, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int d = (int)(i % D);
  const int t = (int)((i / D) % L);
  const int b = (int)(i / ((size_t)D * L));
  const float v = t == 0 ? cls[d] : to_f(patch[((size_t)b * (L - 1) + t - 1) * D + d]);
  tok[i] = from_f<T>(v + pos[(size_t)t * D + d]);
}

template <typename T>
void vit_embed(const void* patch, const float* cls, const float* pos, void* tok, int B, int L,
               int D, hipStream_t st) {
  const size_t n = (size_t)B * L * D;
  vit_embed_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const T*)patch, cls, pos,
                                                                   (T*)tok, L, D, n);
}

template <typename T>
__global__ void rows_to_f32_kernel(const T* x, int ld, float* y, int D, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  y[i] = to_f(x[(i / D) * ld + i % D]);
}

template <typename T>
void rows_to_f32(const void* x, int ld, float* y, int R, int D, hipStream_t st) {
  const size_t n = (size_t)R * D;
  rows_to_f32_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const T*)x, ld, y, D, n);
}

#define INST(T)                                                                               \
  template void unet_prep<T>(const float*, const float*, void*, int, int, int, int, int,      \
                             hipStream_t);                                                    \
  template void unet_out<T>(const void*, int, float*, int, int, int, int, int, hipStream_t);  \
  template void sde_step<T>(int, float*, const float*, const void*, int, int, int,            \
                            const float*, const uint64_t*, uint32_t, StepCoef, int, int, int, \
                            hipStream_t, void*);                                              \
  template void vit_prep<T>(const float*, void*, int, int, hipStream_t);                      \
  template void vit_patches<T>(const float*, void*, int, int, int, hipStream_t);               \
  template void vit_embed<T>(const void*, const float*, const float*, void*, int, int, int,   \
                             hipStream_t);                                                    \
  template void rows_to_f32<T>(const void*, int, float*, int, int, hipStream_t);
INST(float)
INST(bf16)
INST(f16)
#undef INST

// --------------------------------------------------------------------------- text tower
template <typename T>
__global__ void text_embed_kernel(const int64_t* tok, const float* emb, const float* pos, T* x, int N,
                                  int L, int D, int V) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)N * L * D) return;
  const int d = (int)(i % D);
  const size_t nl = i / D;
  const int l = (int)(nl % L);
  const int64_t id = tok[nl];
  const bool ok = id >= 0 && id < V;
  const float v = ok ? emb[(size_t)id * D + d] + pos[(size_t)l * D + d] : __builtin_nanf("");
  x[i] = from_f<T>(v);
}

template <typename T>
void text_embed(const int64_t* tok, const float* emb, const float* pos, void* x, int N, int L, int D, int V,
                hipStream_t st) {
  const size_t n = (size_t)N * L * D;
  text_embed_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(tok, emb, pos, (T*)x, N, L, D, V);
}

// One block per sequence: first position of the largest id (torch.argmax), copy that row.
template <typename T>
__global__ void __launch_bounds__(64) eot_gather_kernel(const int64_t* tok, const T* x, T* out, int L, int D) {
  const int n = blockIdx.x, lane = threadIdx.x;
  int64_t best = INT64_MIN;
  int bi = L;
  for (int l = lane; l < L; l += 64) {
    const int64_t v = tok[(size_t)n * L + l];
    if (v > best) { best = v; bi = l; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  for (int d = lane; d < D; d += 64) out[(size_t)n * D + d] = x[((size_t)n * L + bi) * D + d];
}

template <typename T>
void eot_gather(const int64_t* tok, const void* x, void* out, int N, int L, int D, hipStream_t st) {
  eot_gather_kernel<T><<<N, 64, 0, st>>>(tok, (const T*)x, (T*)out, L, D);
}

// One block (256 threads) per image: cosine scores vs K class texts, x100, softmax, argmax.
__global__ void __launch_bounds__(256) degra_probs_kernel(const float* degra, const float* text, int K,
                                                          int E, float* probs, int32_t* amax) {
  __shared__ float red[8];
  __shared__ float sc[64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* d = degra + (size_t)b * E;
  auto block_sum = [&](float v) {
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  float dd = 0.f;
  for (int e = tid; e < E; e += 256) dd += d[e] * d[e];
  const float dn = sqrtf(block_sum(dd));
  for (int k = 0; k < K; ++k) {
    const float* t = text + (size_t)k * E;
    float tt = 0.f, dt = 0.f;
    for (int e = tid; e < E; e += 256) { tt += t[e] * t[e]; dt += d[e] * t[e]; }
    const float tn = sqrtf(block_sum(tt));
    const float dot = block_sum(dt);
    if (tid == 0) sc[k] = 100.f * (dot / (dn * tn));
  }
  __syncthreads();
  if (tid == 0) {
    float m = -INFINITY;
    int mi = 0;
    for (int k = 0; k < K; ++k)
      if (sc[k] > m) { m = sc[k]; mi = k; }
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += expf(sc[k] - m);
    // argmax over the probabilities themselves (torch.argmax(probs), first maximum).
    float pm = -1.f;
    for (int k = 0; k < K; ++k) {
      const float pk = expf(sc[k] - m) / s;
      probs[(size_t)b * K + k] = pk;
      if (pk > pm) { pm = pk; mi = k; }
    }
    amax[b] = mi;
  }
}

void degradation_probs(const float* degra, const float* text, int B, int K, int E, float* probs,
                       int32_t* argmax, hipStream_t st) {
  degra_probs_kernel<<<B, 256, 0, st>>>(degra, text, K, E, probs, argmax);
}

#define TINST(T)                                                                                 \
  template void text_embed<T>(const int64_t*, const float*, const float*, void*, int, int, int, int, \
                              hipStream_t);                                                      \
  template void eot_gather<T>(const int64_t*, const void*, void*, int, int, int, hipStream_t);
TINST(float)
TINST(bf16)
TINST(f16)
#undef TINST

}  // namespace dac
