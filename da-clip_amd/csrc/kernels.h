// kernels.h — host-side launchers of the gfx950 kernels (one .hip file per family).
// All activations are NHWC ("rows" = pixels/tokens, row stride `ld` elements), stored as
// T = float (parity mode), bf16 (perf mode) or f16 (IEEE half perf mode); small per-image
// vectors are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dac {

enum Act { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_GEGLU = 3 };

// Implicit-GEMM convolution / linear layer:
//   y[m, n] = epi( sum_k A[m, k] * W[n, k] ),  m = (b, oh, ow), k = (kh, kw, ci)
// A gathers the (optionally 2x nearest-upsampled) input; channels [0, C1) come from x1 and
// [C1, Cin) from x2 (fused torch.cat, DenoisingUNet_arch.py:158-161). W is [Cout][KH][KW][Cin].
// Epilogue order (module_util.py:121-129, 143-153): +bias -> *(1+scale)+shift (per image) ->
// act -> +res1 -> +res2 -> +bbias (per image, per channel).
struct ConvArgs {
  const void* x1; const void* x2;
  int ld1, ld2, C1, Cin;
  int Hs, Ws, up;          // source spatial size; up=1: nearest 2x before the conv
  int B, Ho, Wo, Cout, K;
  const void* w;
  const float* bias;       // [Cout] or null
  const float* ss;         // scale [b*ss_ld + n], shift [b*ss_ld + Cout + n]; or null
  int ss_ld;
  const void* res1; int ldr1;
  const void* res2; int ldr2;
  const float* bbias; int bb_ld;   // per-image bias [b*bb_ld + n]; or null
  void* y; int ldy;
  int act;
  // A-loader transform: 0 none; 1 = LinearAttention q path: softmax over each 32-channel
  // head group then * 32^-0.5 (module_util.py:175, 177).
  int amode;
  // > 0: per-image weights W + b * w_bstride (grid.z = B, tiles never straddle images).
  long long w_bstride;
  const void* zero;        // >= 16 zero bytes in global memory (source of padding rows)
  // Row LayerNorm over all Cout channels (gain only, eps ln_eps) applied after bias and before
  // the residual adds: LinearAttention's to_out LayerNorm + Residual (module_util.py:77-86,
  // 180-185). Requires one N tile covering Cout.
  const float* ln_g;
  float ln_eps;
  // Split-precision ("dual") weights of a layer whose bf16 rounding error is systematic enough
  // to move the restored image (engine.cpp Packer::conv dual): W = W_hi + W_lo, stored as the
  // K range [hi | lo] over the input read twice. cwrap > 0: input channel ci >= cwrap reads
  // channel ci - cwrap (two-source layers; then split by C1 as usual); for the 7x7 row-tap
  // layout, kernel row kt >= KH reads row kt - KH.
  int cwrap;
  // Fused second output (the ResBlock's 1x1 res_conv, module_util.py:142,153), 3x3 v4 kernels
  // only: y2[m, n] = sum_c x[m @ centre tap, c] * w2[n, c] (+ bias2), over the same (x1 | x2)
  // input the conv reads; w2 is [Cout][Cin] bf16, or [Cout][hi Cin | lo Cin] with w2_dual.
  const void* w2;
  const float* bias2;
  int w2_dual;
  void* y2; int ldy2;
  // Row LayerNorm of the INPUT folded into a 1x1 GEMM (SpatialTransformer norm1 -> q|k|v and
  // norm3 -> GEGLU proj, attention.py:253-261): the weights are pre-multiplied by the LN gain
  // (w = W diag(g)), bias = b + W beta, and the kernel takes the row moments of x from its own
  // A fragments, then y = rstd * (x.w^T - mean * lnf_cs[n]) + bias with lnf_cs[n] = sum_k w[n][k]
  // (of the stored, rounded weights). lnf_n = channels in the mean, lnf_eps the LN epsilon.
  const float* lnf_cs;
  int lnf_n;
  float lnf_eps;
  // GroupNorm of the INPUT applied in a 1x1 GEMM's A path (SpatialTransformer norm ->
  // proj_in, attention.py:76-77, 239-241): the A fragments are mapped x -> x * s + t per
  // channel, s = rstd(b, g) * gamma, t = beta - mean(b, g) * s, rounded back to T (what a
  // separate GroupNorm pass would have stored). gna_nb == 0: gna_stats = [B][groups][mean,
  // rstd]; gna_nb > 0: gna_stats = [B][groups][gna_nb][sum, sum of squares] per-block sums of
  // the PreNorm LayerNorm kernel (layernorm_gnstats), merged by every block in fixed order with
  // eps gna_eps.
  const float* gna_stats;
  const float* gna_g;
  const float* gna_b;
  int gna_groups;
  // Set by the dispatcher, never by callers: the 1x1 GEMM kernels (conv2_kernel) issue their
  // LDS-DMA through buffer descriptors (one row pitch, 31-bit byte offsets).
  int dbuf;
  int gna_nb;
  float gna_eps;
  // fp8 (OCP e4m3) activations with one E8M0 exponent per (pixel, 32-channel half): the fp8
  // handles' ResBlock-internal tensor h between block1 and block2 (module_util.py:143-153),
  // written by block1's epilogue and read only by block2's conv (conv3q.hip).
  //   ys8 != null: the epilogue writes y as e4m3 bytes (ldy in bytes) and the exponents of pixel
  //   m to ys8[m * (Cout / 32) + n / 32] (value = e4m3 * 2^(ys8 - 127)).
  //   xs8: the exponents of an e4m3 input x1 (ld1 in bytes), same layout.
  uint8_t* ys8;
  const uint8_t* xs8;
  // Row-phase form of a 3x3 conv over a 2x nearest-upsampled input (up = 1; the UNet's
  // Upsample, module_util.py:100-103): output row 2i+a reads source rows (i-1, i, i) for a = 0
  // and (i, i, i+1) for a = 1, so its three kernel rows collapse to two with summed weights.
  // uph = 1: w is [Cout][4 rows][3][Cin] = (W0, W1+W2 | W0+W1, W2), K = 12 Cin, and the v4 tiles
  // hold output rows of one parity (2 kernel-row stages per chunk instead of 3). uph = 2: the
  // columns fold the same way (each wave one column parity, 2 taps over source pixels):
  // w is [Cout][4 row sets][4 (column parity, tap)][Cin], K = 16 Cin (rows >= 128 pixels).
  int uph;
  // Split-K (1x1 GEMMs whose tile grid leaves the chip idle: the ViT / text linears, M = B x L):
  // ksplit > 1 blocks along grid z each sum a contiguous range of K tiles into part
  // [ksplit][M][Cout] (fp32, no epilogue); conv_part_reduce then sums them in fixed order and
  // applies the epilogue (bias, activation, residuals) — set by the engine with the workspace.
  int ksplit;
  float* part;
  // GEGLU projections (attention.py:37-64), 16-bit: the same weights in the swapped-tile order
  // (w_gs, bias b_gs): in each 64-row group G, rows 16 lg + e hold the x rows (e < 8) and the gate
  // rows (e >= 8) of output channels 32 G + 8 lg + (e & 7), so a swapped tile's lane ends with x
  // and gate of 8 consecutive output channels of one pixel (register epilogue, 16-byte stores).
  // Null: only the 16-row-interleaved order in w / bias exists.
  const void* w_gs;
  const float* b_gs;
  // In-graph launch timing (bench roofline, engine Profiler::stamps): null, or a [begin, end]
  // pair of 64-bit device words: the kernel's first wave atomic-mins its start and every wave
  // atomic-maxes its end on the constant-rate wall clock (common.h StampGuard).
  unsigned long long* stamp;
};
// The dispatcher has an LN-folding kernel for this 1x1 GEMM (16-bit types only).
bool conv_lnf_ok(const ConvArgs& a, int elem_bytes);
// ... and a kernel applying the input GroupNorm in its A path (ConvArgs::gna_stats).
bool conv_gna_ok(const ConvArgs& a, int elem_bytes);
// GroupNorm statistics only (norm.hip): the (mean, rstd) table groupnorm() applies, at
// part + B * groups * GN_CHUNKS * 3 (returned).
template <typename T>
const float* groupnorm_stats(const void* x, int B, int HW, int C, int groups, float eps, float* part,
                             hipStream_t st);
// LayerNorm whose output also yields that tensor's GroupNorm statistics (norm.hip): per-block
// group sums [B][groups][nb][sum, sum of squares] into part; returns nb (blocks per image), or 0
// if the shape is not covered; launch = false only answers.
template <typename T>
int layernorm_gnstats(const void* x, int ldx, void* y, int ldy, const float* g, const float* b, int rows, int C,
                      float eps, int HW, int groups, float* part, bool launch, hipStream_t st);
size_t layernorm_gnstats_ws_floats(int B, int HW, int groups);
// The dispatcher can fuse a_w2/y2 into this 3x3 conv (bf16 v4 256x64 swapped-operand tiles).
bool conv_res_fusable(const ConvArgs& a);

// Shapes served by the weight-stationary 3x3 kernel (conv_impl.h conv3w_kernel, 16-bit types).
inline bool conv3w_ok(const ConvArgs& a) {
  return a.Cin == 64 && a.Cout == 64 && a.K == 576 && a.cwrap == 0 && !a.y2 && (!a.ss || (a.ss_ld % 4 == 0 && ((uintptr_t)a.ss & 15) == 0)) && a.zero && a.amode == 0 && a.w_bstride == 0 &&
         !a.ln_g && (a.act == ACT_NONE || a.act == ACT_SILU) && a.Wo >= 64 && a.Wo % 64 == 0 &&
         (a.C1 >= a.Cin || a.C1 % 32 == 0) && a.ldy % 8 == 0 && a.ld1 % 8 == 0 &&
         (a.C1 >= a.Cin || a.ld2 % 8 == 0) && (!a.res1 || a.ldr1 % 8 == 0) && !a.res2 && !a.bbias && !(a.ss && a.res1);   // (epi_regs16 PRE)
}
template <typename T>
void conv(const ConvArgs& a, int kh, int kw, int stride, int pad, hipStream_t st);
// Fused ResBlock (rbfuse.hip, 16-bit types; module_util.py:132-153): block1 (3x3 Cin -> 64,
// per-image scale / shift, SiLU) and block2 (3x3 64 -> 64, SiLU) + residual in one launch, h (and
// the 1x1 res_conv output) never leaving LDS. Cin = 64 (residual = x) or 128 (x1 | x2 = torch.cat
// of two 64-channel tensors, or one 128-channel tensor; residual = x w_res^T).
struct RbArgs {
  const void* x1; const void* x2;
  int ld1, ld2, C1, Cin;
  int B, H, W;
  const void* w1;          // [64][3][3][Cin]
  const void* w2;          // [64][3][3][64]
  const void* wr;          // [64][Cin] (Cin = 128) or null
  const float* ss; int ss_ld;    // scale [b * ss_ld + n], shift [b * ss_ld + 64 + n]
  void* y; int ldy;
  unsigned long long* stamp;     // in-graph launch timing, as ConvArgs::stamp
};
bool rbfuse_pays(const RbArgs& a);
bool rbfuse_ok(const RbArgs& a);
template <typename T>
void rbfuse(const RbArgs& a, hipStream_t st);
// Register-stationary 3x3 conv, 64 -> 64 (conv3r.hip, 16-bit types): the shapes it serves
// (DAC_CONV3R=0 turns it off) and its launcher.
bool conv3r_ok(const ConvArgs& a);
template <typename T>
void conv3r(const ConvArgs& a, hipStream_t st);
// init_conv (7x7, Cin 8 row-tap layout, Cout 64, bf16 / f16, plain or split-precision weights):
// weight-stationary persistent kernel (conv_edge.hip).
bool conv7_ok(const ConvArgs& a);
// v6 2-D halo 3x3 kernel (conv_impl.h conv3h_kernel) takes this conv (conv.hip).
bool conv3h_ok(const ConvArgs& a, int elem_bytes);
template <typename T>
void conv7(const ConvArgs& a, hipStream_t st);
// final_conv (3x3, Cin 64 -> Cout <= 4, bf16 / f16, plain or split-precision weights, Wo % 64 == 0):
// streaming kernel with hi/lo as separate MFMA rows (conv_edge.hip).
bool conv3n_ok(const ConvArgs& a);
template <typename T>
void conv3n(const ConvArgs& a, hipStream_t st);
// Downsample (4x4, stride 2, pad 1, bf16 / f16, Cin % 32 == 0, Cout % 64 == 0): row-band tiles with
// deinterleaved even / odd input pixels (conv_down.hip).
bool conv_down_ok(const ConvArgs& a);
template <typename T>
void conv_down(const ConvArgs& a, hipStream_t st);
int conv_variant(const ConvArgs& a, int kh, int elem_bytes);

// fp8 (e4m3, MX block scales) implicit GEMM for bf16 / fp16 activations (conv8.hip): w8 [Cout][Kp]
// e4m3 weights (K padded to Kp, a multiple of 128, with zeros), ws8 [Cout][Kp / 64] E8M0
// exponents (weight = w8 * 2^(ws8 - 127)). conv8_ok: shapes / layouts it serves.
bool conv8_ok(const ConvArgs& a, int kh, int kw, int s, int p);
template <typename T>
void conv8(const ConvArgs& a, int kh, int kw, int s, int p, const uint8_t* w8, const uint8_t* ws8, int Kp,
           hipStream_t st);
// fp8 ResBlock pair (conv3q.hip). Producer: a 3x3 conv with ys8 set (block1, 16-bit input) whose
// epilogue writes e4m3 + exponents; conv_q8out_ok says the dispatcher has such a kernel for it
// (the weight-stationary 64 -> 64 conv, or the fused-res_conv v4 tiles with Cout = 64).
// Consumer: block2's 3x3 conv 64 -> 64 over that e4m3 input (x1, xs8, ld1 = 64 bytes) with
// weight-stationary e4m3 weights q8w [64 out][9 taps][64 in] and exponents q8s [64][9][2]
// (per output channel, tap and 32-channel half), on the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4; 16-bit output with the conv3w epilogue (bias, SiLU, res1).
bool conv_q8out_ok(const ConvArgs& a);
// Split-K (ConvArgs::ksplit / part): the 1x1 GEMM this engine call would split, and its second
// pass (sum of the ksplit partials in order, then bias -> scale/shift -> activation -> residuals).
int conv_split_k(const ConvArgs& a, int elem_bytes, long rows);
// 3x3 (stride 1, pad 1) split-K: the v3 form can take this conv with ksplit > 1 (plain
// epilogues: bias, scale/shift, SiLU, residuals; no fused res_conv, upsampling, fp8 or phases).
bool conv3_split_ok(const ConvArgs& a, int elem_bytes);
// Split count of such a conv from ONE image's shape: `ks` Cin ranges of >= 2 chunks each.
int conv3_split_k(const ConvArgs& a, int elem_bytes, int ks);
template <typename T>
void conv_part_reduce(const ConvArgs& a, hipStream_t st);
// Row-phase upsample conv (ConvArgs::uph): the dispatcher has the kernel for this conv.
bool conv_uph_ok(const ConvArgs& a);
bool conv3q_ok(const ConvArgs& a);
template <typename T>
void conv3q(const ConvArgs& a, const uint8_t* q8w, const uint8_t* q8s, hipStream_t st);

// Row LayerNorm over C (channel LN of NHWC == token LN):
//   y = [res +] (x - mean) * rsqrt(var + eps) * g [+ b]
template <typename T>
void layernorm(const void* x, int ldx, void* y, int ldy, const void* res, int ldr,
               const float* g, const float* b, int rows, int C, float eps, hipStream_t st);

// GroupNorm(groups, eps, affine) on NHWC [B, HW, C] -> y (same layout).
template <typename T>
void groupnorm(const void* x, void* y, const float* g, const float* b, int B, int HW, int C,
               int groups, float eps, float* stats_ws, hipStream_t st);

// Multi-head self-attention over rows of qkv [B*L, 3*H*D] (q | k | v), D = 32 (UNet
// SpatialTransformer, attention.py:170-193) -> o [B*L, H*D].
template <typename T>
void flash_attn_d32(const void* qkv, void* o, int B, int L, int H, float scale, hipStream_t st);
// variant 1 forces the staged-tile kernel for this call (op-level test hook).
template <typename T>
void flash_attn_d32_v(const void* qkv, void* o, int B, int L, int H, float scale, int variant, hipStream_t st);
extern int g_flash_old;

// CLIP text tower helpers: token + positional embedding gather (ids outside [0, V) -> NaN),
// EOT-row gather (position of the highest id per sequence), degradation-class scoring.
template <typename T>
void text_embed(const int64_t* tok, const float* emb, const float* pos, void* x, int N, int L, int D, int V,
                hipStream_t st);
template <typename T>
void eot_gather(const int64_t* tok, const void* x, void* out, int N, int L, int D, hipStream_t st);
void degradation_probs(const float* degra, const float* text, int B, int K, int E, float* probs,
                       int32_t* argmax, hipStream_t st);

// nn.MultiheadAttention core for short sequences (ViT / CLIP text), head dim D = 64, any L;
// causal != 0 applies the text tower's causal mask.
template <typename T>
void small_mha(const void* qkv, void* o, int B, int L, int H, int D, int causal, hipStream_t st);

// LinearAttention (module_util.py:170-185) context on qkv [B*HW, 384] (q | k | v):
//   la_kmax   : per (image, chunk) channel max of k
//   la_ctx    : per (image, chunk) sum_n exp(k - max) v^T on MFMA (+ exp sums)
//   la_reduce : merge chunk partials in fixed order (deterministic)
//   la_weff   : W_eff[b][c][h*32+d] = sum_e Wout[c][h*32+e] ctx[b][h][d][e] / sum / HW
// The to_out 1x1 conv then runs as a GEMM of softmax_d(q)*scale (fused into its A loader,
// amode = 1) with the per-image W_eff: Wout (ctx^T q) = (Wout ctx^T) q.
// hw_scale > 0 replaces the 1/HW factor of W_eff (f16: W_eff / HW is subnormal, so the caller
// stores W_eff * S / HW and scales the GEMM's accumulators by 1/S, S a power of two).
template <typename T>
void linear_attention_weff(const void* qkv, const float* wout, void* weff, int B, int HW, int C,
                           float* ws, hipStream_t st, float hw_scale = 0.f);
// Whole LinearAttention block, Residual(PreNorm(LinearAttention)) (module_util.py:27-33,
// 89-97, 157-185), for C in {64, 128, 256}: y = x + LN_out(to_out(ctx^T softmax_d(q))) with the
// to_out bias and gain; wqkv: to_qkv [384][C] with the PreNorm gain folded in (w diag(g));
// weff: [B][C][128] scratch (per-image to_out weights), ws: linear_attention_fused_ws_floats(B, HW)
// floats; qshift > 0: a bound on every |q| of the layer, used as the q-softmax shift (0: per-pixel max).
template <typename T>
void linear_attention_fused(const void* x, const void* wqkv, const float* wout, const float* bout,
                            const float* gout, void* weff, void* y, int B, int HW, int C, float* ws,
                            hipStream_t st, float qshift = 0.f);
size_t linear_attention_fused_ws_floats(int B, int HW);
size_t linear_attention_ws_floats(int B, int HW);

// Small fp32 dense layer for per-image vectors (time / prompt MLPs, ViT head):
//   y[r, o] = post( b[o] + sum_i pre(x[r*ldx + i]) * W[o*I + i] ) (+ add[r % add_mod, o])
void small_linear(const float* x, int ldx, const float* W, const float* b, float* y, int ldy,
                  int R, int I, int O, int pre_act, int post_act, const float* add, int add_ld,
                  int add_mod, hipStream_t st);
// out[r, :nf] = SinusoidalPosEmb(float((t0 + dt * (r / B)) * scale)) for r < R
// (module_util.py:41-48; scale = IRSDE.sample_scale).
void sinus_embedding(float* out, int R, int B, int nf, double t0, double dt, double scale,
                     hipStream_t st);
// Precision analysis: y[r*ld + c] = float(bf16(y[r*ld + c])) for r < rows, c < C (or the
// fp16 rounding with DAC_EMU_FP16=1).
void round_bf16_rows(float* y, int ld, size_t rows, int C, hipStream_t st);
// One shared (scale, shift) row for a conv epilogue: ss[0:C] = scale_m1, ss[C:2C] = shift[c]
// (read with ss_ld = 0 by every image).
void ss_fill(float* ss, int C, float scale_m1, const float* shift, hipStream_t st);
// p[0] = a, p[1] = b on the device, in stream order.
void set_u64x2(uint64_t* p, uint64_t a, uint64_t b, hipStream_t st);
// n [begin, end] stamp pairs reset to [UINT64_MAX, 0] (ConvArgs::stamp, engine Profiler).
void stamp_init(unsigned long long* s, size_t n, hipStream_t st);
// y[r, :] = softmax(x[r, :]) * v  (DenoisingUNet_arch.py:134)
void softmax_mul(const float* x, const float* v, float* y, int R, int C, hipStream_t st);

// UNet input: x[b, h, w, 0:8] = (xt - mu, mu, 0, 0) with reflect padding to (Hp, Wp)
// (DenoisingUNet_arch.py:123-127). xt, mu: NCHW fp32 [B, 3, H, W].
template <typename T>
void unet_prep(const float* xt, const float* mu, void* x, int B, int H, int W, int Hp, int Wp,
               hipStream_t st);

// Crop the padded NHWC model output (channels [0,3) of rows of stride ld) to NCHW fp32.
template <typename T>
void unet_out(const void* y, int ld, float* eps, int B, int H, int W, int Hp, int Wp,
              hipStream_t st);

// Sampler updates on NCHW fp32 state (sde_utils.py:205-231, 245-247 / 44-45, 177-187).
// eps is the padded NHWC model output. z: explicit noise or null -> Philox(*seedp, tag).
// xin (loop form only, unpadded images): also write the next step's UNet input there, exactly
// as unet_prep would from the new x (so the next forward skips its unet_prep launch).
struct StepCoef { float sbar, ea, t1, t2, std, theta, sigma2, dt, sigma_sqrt_dt; };
template <typename T>
void sde_step(int mode, float* x, const float* mu, const void* eps, int ld, int Hp, int Wp,
              const float* z, const uint64_t* seedp, uint32_t tag, StepCoef c, int B, int H,
              int W, hipStream_t st, void* xin = nullptr);
// Whether sde_step can take xin for this layout (the per-pixel kernel on unpadded images).
bool sde_step_fuses(int ld, int H, int W, int Hp, int Wp);

// ViT input: NCHW fp32 image -> NHWC T with channels padded to VE.
template <typename T>
void vit_prep(const float* img, void* x, int B, int S, hipStream_t st);
// ViT stem input as GEMM rows: [B * (S/P)^2][3 P P] in (ky, kx, c) order (stride == kernel).
template <typename T>
void vit_patches(const float* img, void* x, int B, int S, int P, hipStream_t st);
// tokens[b, 0] = cls + pos[0]; tokens[b, 1+p] = patch[b, p] + pos[1+p]
template <typename T>
void vit_embed(const void* patch, const float* cls, const float* pos, void* tok, int B, int L,
               int D, hipStream_t st);
// Gather row 0 of each image's tokens to fp32 [B, D] (after ln_post).
template <typename T>
void rows_to_f32(const void* x, int ld, float* y, int R, int D, hipStream_t st);

}  // namespace dac
