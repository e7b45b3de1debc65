/*
 * daclip_hip.h — C ABI of libdaclip_hip.so, the MI355X-native DA-CLIP + IR-SDE hot path.
 *
 * The reference (yeeecheng/DA-CLIP) has no native plugin API; its plug points are Python
 * callables. Each entry point below replaces one of them:
 *
 *   dac_create / dac_set_weight / dac_finalize_weights
 *       replace module construction + strict `load_state_dict`:
 *       open_clip/factory.py:99-106 (load_checkpoint), factory.py:365-404
 *       (create_model_from_pretrained), config/daclip-sde/models/base_model.py:92-105
 *       (load_network) and networks.py:10-15 (define_G -> ConditionalUNet(**setting)).
 *   dac_encode_image
 *       replaces DaCLIP.encode_image(image, control=True)   (open_clip/daclip_model.py:46-53)
 *       and, with degra_ctx NULL, encode_image(image, control=False) (daclip_model.py:54-55)
 *   dac_encode_text / dac_degradation_probs
 *       replace DaCLIP.encode_text (daclip_model.py:125-126 -> model.py:237-249) and the
 *       degradation-class scoring softmax(100 d^ t^T) -> argmax (evaluate_daclip.py:45-84)
 *   dac_unet_forward
 *       replaces the `sde.set_model(model)` callable: model(x, mu, t, text_context=,
 *       image_context=) -> noise (utils/sde_utils.py:163-164, 195-202;
 *       DenoisingUNet_arch.py:118-174)
 *   dac_sde_schedule
 *       replaces IRSDE._initialize                          (utils/sde_utils.py:84-154)
 *   dac_sde_reverse
 *       replaces IRSDE.reverse_posterior / reverse_sde      (utils/sde_utils.py:261-313)
 *       as one hipGraph-captured loop
 *   dac_posterior_step
 *       replaces IRSDE.reverse_posterior_step / reverse_sde_step (sde_utils.py:44-45, 227-231)
 *
 * Conventions: every tensor argument is a caller-owned DEVICE pointer to contiguous fp32
 * NCHW data (torch `data_ptr()`), on the handle's device. `stream` is a hipStream_t (NULL =
 * default stream). Functions return 0 on success and a negative DAC_E* code on error; the
 * message is available from dac_last_error(). A handle owns its weights, workspace and
 * graphs; calls on one handle must be serialised; handles on different devices are
 * independent (one handle per GPU / rank).
 */
#ifndef DACLIP_HIP_H
#define DACLIP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dac_handle dac_handle;

/* compute/storage dtype. DAC_FP8 (BASELINE configs[4]): bf16 activations and kernels, with
 * the block-scaled fp8 MFMA where its operands arrive as OCP e4m3 without VALU work: the UNet's
 * 64 -> 64 ResBlock block2 convs read the e4m3 tensor (one E8M0 exponent per pixel and 32
 * channels) that block1's epilogue writes, with e4m3 weights (one exponent per output channel,
 * tap and 32 input channels); the ViT's GEMMs take e4m3 weights (one exponent per 64 k).
 * DAC_F16: IEEE half weights and activations on the f16 MFMA, fp32 accumulate — the same
 * bytes and MFMA rate as DAC_BF16 with an 11-bit instead of 8-bit significand. */
enum dac_dtype { DAC_F32 = 0, DAC_BF16 = 1, DAC_FP8 = 2, DAC_F16 = 3 };
enum dac_src_dtype { DAC_SRC_F32 = 0, DAC_SRC_F16 = 1, DAC_SRC_BF16 = 2 };
enum dac_mode { DAC_POSTERIOR = 0, DAC_SDE = 1 };       /* DenoisingModel.test(mode=) */
enum dac_schedule { DAC_COSINE = 0, DAC_LINEAR = 1, DAC_CONSTANT = 2 };

enum dac_err {
  DAC_OK = 0,
  DAC_E_ARG = -1,        /* bad argument / shape / dtype */
  DAC_E_KEY = -2,        /* unknown state_dict key or shape mismatch */
  DAC_E_MISSING = -3,    /* dac_finalize_weights: required key never set (strict load) */
  DAC_E_STATE = -4,      /* call order (e.g. forward before finalize) */
  DAC_E_HIP = -5,        /* HIP runtime error */
  DAC_E_NOMEM = -6
};

/* Network configuration. UNet fields mirror options/test.yml network_G.setting
 * (DenoisingUNet_arch.py:22-23); vision fields mirror CLIPVisionCfg
 * (open_clip/model_configs/daclip_ViT-B-32.json). Zero `unet`/`vit` skips that network. */
typedef struct dac_config {
  int unet;
  int in_nc, out_nc, nf, depth, ch_mult[8], context_dim;
  int use_degra_context, use_image_context;
  int vit;
  int image_size, patch_size, width, layers, head_width, mlp_width, embed_dim;
  /* Text tower (CLIPTextCfg, open_clip/model_configs/daclip_ViT-B-32.json text_cfg); needs vit.
   * Zero `text` leaves it out (its checkpoint keys are then accepted and ignored). */
  int text;
  int context_length, vocab_size, text_width, text_heads, text_layers;
  /* Wild-IR UNet variant (config/wild-ir/models/modules/DenoisingUNet_arch.py:22-40):
   * unet_scale_half = 1 for `scale: 0.5` (extra Downsample/Upsample around the levels);
   * unet_st_from = first level with a SpatialTransformer (0 = 3, the daclip-sde rule). */
  int unet_scale_half, unet_st_from;
} dac_config;

int dac_create(int device, int dtype, const dac_config* cfg, dac_handle** out);
void dac_destroy(dac_handle* h);

/* Copy one reference state_dict tensor (host or device pointer) into the handle,
 * repacking it to the kernel layout. Keys use the reference names, e.g.
 * "downs.0.0.block1.proj.weight", "clip.visual.transformer.resblocks.0.attn.in_proj_weight",
 * "visual_control.transformer.zero_modules.0.weight". Keys the hot path does not use
 * (text tower, logit_scale) are accepted and ignored (returns 1). */
int dac_set_weight(dac_handle* h, const char* key, const void* data, const int64_t* shape,
                   int ndim, int src_dtype);
/* Strict check: every key the configured networks need was set. */
int dac_finalize_weights(dac_handle* h);

/* img [B,3,S,S] (preprocessed, S = image_size) -> image_ctx [B,E], degra_ctx [B,E] fp32.
 * degra_ctx NULL runs DaCLIP.encode_image(image, control=False) instead
 * (open_clip/daclip_model.py:54-55 -> CLIP.encode_image, model.py:233-235): the clip tower
 * alone, no controller hiddens, its features in image_ctx. */
int dac_encode_image(dac_handle* h, const float* img, int B, float* image_ctx,
                     float* degra_ctx, void* stream);

/* Text features (CLIP.encode_text, open_clip/model.py:237-249, via DaCLIP.encode_text
 * daclip_model.py:125-126): tokens [N, context_length] int64 device ids (open_clip.tokenize
 * output) -> text_features [N, embed_dim] fp32, unnormalised. Ids outside the vocabulary give
 * NaN features (never an out-of-bounds read). */
int dac_encode_text(dac_handle* h, const int64_t* tokens, int N, float* text_features, void* stream);

/* Degradation-class scoring (evaluate_daclip.py:45-50, 78-84): probs[B][K] =
 * softmax_k(100 * <degra_b / |degra_b|, text_k / |text_k|>), argmax[B] = first maximum.
 * degra [B, E], text_features [K, E] fp32 device; K <= 64. */
int dac_degradation_probs(dac_handle* h, const float* degra, const float* text_features, int B, int K,
                          int E, float* probs, int32_t* argmax, void* stream);

/* One ConditionalUNet forward: eps = model(xt, mu, t, text_ctx, image_ctx), all [B,3,H,W]
 * except contexts [B,context_dim]; text_ctx / image_ctx may be NULL. */
int dac_unet_forward(dac_handle* h, const float* xt, const float* mu, float t,
                     const float* text_ctx, const float* image_ctx, int B, int H, int W,
                     float* eps_out, void* stream);

/* IR-SDE schedule. If `tables` is non-NULL it holds 4*(T+1) host floats
 * [thetas | sigmas | thetas_cumsum | sigma_bars] computed by the caller (bit-identical to the
 * reference's torch ops) and `dt` is used as given; otherwise the tables are computed here
 * in fp32 following sde_utils.py:91-154. */
int dac_sde_schedule(dac_handle* h, float max_sigma, int T, int schedule, float eps,
                     const float* tables, float dt);

/* Full reverse loop t = T..1 in place on x_inout [B,3,H,W] with mu = LQ [B,3,H,W].
 * noise: NULL -> device Philox N(0,1) keyed by (seed, step, element); else [T,B,3,H,W]
 * fp32 device tensor, slice i consumed at step t = T - i (parity mode). Captured once per
 * (B,H,W,T,mode, which contexts / noise are given) as a hipGraph and replayed; injected
 * noise is copied into a handle-owned buffer first, so the caller may free or reuse it.
 * text_ctx NULL skips the prompt embedding (DenoisingUNet_arch.py:133-137); image_ctx NULL
 * makes every SpatialTransformer's attn2 a self-attention (attention.py:174), which, as in
 * the reference, requires context_dim == channels at those levels (DAC_E_ARG otherwise). */
int dac_sde_reverse(dac_handle* h, int mode, float* x_inout, const float* mu,
                    const float* text_ctx, const float* image_ctx, int B, int H, int W, int T,
                    const float* noise, uint64_t seed, void* stream);

/* Device-noise keying for sharded runs: with noise == NULL, element e of image b draws
 * Philox(seed, step, (first_image + b) * 3*H*W + e), so a shard whose first global image is
 * `first_image` reproduces exactly the noise that image receives in an unsharded batch
 * (results are independent of the world size). Default 0. */
int dac_set_noise_offset(dac_handle* h, uint64_t first_image);

/* Time fed to the model at step t: t * scale, with scale = IRSDE.sample_scale = T / sample_T
 * (utils/sde_utils.py:86-88, 266, 302: noise_fn(x, t, self.sample_scale)). Default 1. The
 * product is formed in double and rounded once to float32, like the reference's python float
 * becoming torch.tensor([time]) (DenoisingUNet_arch.py:120-121). */
int dac_sde_set_time_scale(dac_handle* h, double scale);

/* One sampler update given the model output: x <- step(x, eps, t, z); x, eps, mu, z are
 * [B,3,H,W] fp32 and n = B*3*H*W elements (must be a multiple of 3). */
int dac_posterior_step(dac_handle* h, int mode, float* x_inout, const float* eps,
                       const float* mu, const float* z, int t, int n, void* stream);

/* Workload model: algorithmic FLOPs of one UNet forward at (B,H,W) and of one encode,
 * counted 2*MAC over conv/linear/bmm like torch.utils.flop_counter. */
double dac_unet_flops(dac_handle* h, int B, int H, int W);
double dac_encode_flops(dac_handle* h, int B);

/* Kernel timing over the next dac_sde_reverse call: HIP events around every launch of
 * the dominant conv class (`kernel_id` = 0), on the stream it runs on. Returns the
 * number of timed launches and their mean duration (ms) / flops per launch. */
int dac_profile_enable(dac_handle* h, int kernel_id);
int dac_profile_read(dac_handle* h, double* mean_ms, double* flops_per_launch,
                     double* bytes_per_launch);
/* graph_stamps = 1: the profiled dac_sde_reverse records its loop into a captured graph exactly
 * as the timed loop (side-stream branches included) with a wall-clock [begin, end] stamp pair
 * written by every launch of the class (kernel_id 999 = every conv launch), replays it once and
 * reads each launch's in-graph duration (HIP events cannot be timed inside graph replays);
 * 0 (default) = the eager replay with an event pair around each launch. */
int dac_profile_mode(dac_handle* h, int graph_stamps);
/* Launch i of the last profile (after dac_profile_read): duration (ms), algorithmic flops and
 * bytes, conv class (kh*100 + variant), (graph mode) start time in ms after the replay's first
 * profiled launch (-1 in eager mode), whether it ran in a concurrent branch of the UNet's split
 * section, its shape label and (graph mode) the kernel symbol. */
int dac_profile_launch(dac_handle* h, int i, double* ms, double* flops, double* bytes, int* kernel_class,
                       double* start_ms, int* in_branch, char* label, int label_len, char* symbol,
                       int symbol_len);
/* Graph mode: HIP-event time (ms) of the profiled graph replay on the loop's stream. */
int dac_profile_graph_ms(dac_handle* h, double* ms);

/* Op-level test hook: the SpatialTransformer self-attention core on its own (the kernel
 * dac_unet_forward runs for attention.py:170-193). qkv is [B*L, 3*H*32] (q | k | v, heads
 * of 32), out [B*L, H*32], both in `dtype` (DAC_F32 / DAC_BF16) on the current device;
 * scale = 32^-0.5. variant: 0 = the dispatcher's choice, 1 = the staged-tile kernel,
 * 2 = the K/V-ring kernel (16-bit dtypes, L % 64 == 0; DAC_E_ARG otherwise), 3 = the 16-wave
 * K/V-resident kernel (16-bit dtypes, L % 256 == 0, L <= 1024; DAC_E_ARG otherwise), 4 = the
 * same with its two query groups per wave walked jointly (prescaled q and L % 512 == 0; other
 * shapes run as 3; same constraints as 3).
 * variant | DAC_ATTN_Q_PRESCALED: q was multiplied by 32^-0.5 * log2(e) before rounding (as the
 * 16-bit handles' q|k|v weights are), so scores come out in log2 units.
 * dtype: DAC_F32, DAC_BF16 or DAC_F16. */
enum { DAC_ATTN_Q_PRESCALED = 8 };
int dac_op_attention(const void* qkv, void* out, int B, int L, int H, int dtype, int variant,
                     void* stream);

const char* dac_last_error(dac_handle* h);

/* Build provenance baked in at compile time: "<sha256 of the library sources>[:16] git=<HEAD>"
 * (da-clip_amd/Makefile). The Python side recomputes the source hash from the tree, so a run
 * can prove which sources the loaded library was built from. */
const char* dac_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* DACLIP_HIP_H */
