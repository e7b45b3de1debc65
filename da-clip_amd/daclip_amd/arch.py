"""Architecture configs and state_dict layouts for the two networks on the hot path.

The key names and shapes reproduce the reference modules exactly so that released
checkpoints load unchanged:

* ConditionalUNet — universal-image-restoration/config/daclip-sde/models/modules/
  DenoisingUNet_arch.py:22-109 (blocks from module_util.py:100-185, attention.py:152-261).
* DaCLIP vision towers — open_clip/daclip_model.py:17-24, open_clip/transformer.py:189-555,
  open_clip/model.py:86-145 (VisionTransformer with nn.GELU + LayerNorm, head_width 64).

tests/test_arch.py checks these layouts against tests/golden/state_spec.json, which was
dumped from the reference modules themselves.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

Shape = Tuple[int, ...]


@dataclass(frozen=True)
class UNetConfig:
    """`network_G.setting` of options/test.yml:30-39 (universal-ir)."""
    in_nc: int = 3
    out_nc: int = 3
    nf: int = 64
    ch_mult: Tuple[int, ...] = (1, 2, 4, 8)
    context_dim: int = 512
    use_degra_context: bool = True
    use_image_context: bool = True
    # Wild-IR (config/wild-ir/models/modules/DenoisingUNet_arch.py:22-40, 136-140, 176-180):
    # scale == 0.5 adds Downsample(nf, nf) after init_conv and Upsample(nf, nf) before the
    # final concat; SpatialTransformer levels start at depth - 1 there, at 3 in daclip-sde.
    scale: float = 1.0
    st_from: int = 3

    @property
    def depth(self) -> int:
        return len(self.ch_mult)

    @property
    def time_dim(self) -> int:
        return self.nf * 4

    def levels(self) -> List[Tuple[int, int]]:
        """(dim_in, dim_out) per level, DenoisingUNet_arch.py:67-71."""
        m = (1,) + tuple(self.ch_mult)
        return [(self.nf * m[i], self.nf * m[i + 1]) for i in range(self.depth)]

    def uses_transformer(self, level: int) -> bool:
        """SpatialTransformer vs LinearAttention selection, DenoisingUNet_arch.py:78-83."""
        return self.use_image_context and self.context_dim > 0 and level >= self.st_from


@dataclass(frozen=True)
class VisionConfig:
    """CLIPVisionCfg fields used by daclip_ViT-B-32.json (open_clip/model.py:25-50)."""
    image_size: int = 224
    patch_size: int = 32
    width: int = 768
    layers: int = 12
    head_width: int = 64
    mlp_ratio: float = 4.0
    embed_dim: int = 512

    @property
    def heads(self) -> int:
        return self.width // self.head_width

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def tokens(self) -> int:
        return self.grid * self.grid + 1


@dataclass(frozen=True)
class TextConfig:
    context_length: int = 77
    vocab_size: int = 49408
    width: int = 512
    heads: int = 8
    layers: int = 12


VIT_B_32 = VisionConfig()
VIT_L_14 = VisionConfig(patch_size=14, width=1024, layers=24, embed_dim=768)
TEXT_B_32 = TextConfig()
TEXT_L_14 = TextConfig(width=768, heads=12)

MODEL_CONFIGS: Dict[str, Tuple[VisionConfig, TextConfig]] = {
    "daclip_ViT-B-32": (VIT_B_32, TEXT_B_32),
    "daclip_ViT-L-14": (VIT_L_14, TEXT_L_14),
}


# ----------------------------------------------------------------------------- UNet

def _resblock(p: str, din: int, dout: int, tdim: int, sd: "OrderedDict[str, Shape]"):
    # module_util.py:132-153
    sd[p + "mlp.1.weight"] = (dout * 2, tdim)
    sd[p + "mlp.1.bias"] = (dout * 2,)
    sd[p + "block1.proj.weight"] = (dout, din, 3, 3)
    sd[p + "block2.proj.weight"] = (dout, dout, 3, 3)
    if din != dout:
        sd[p + "res_conv.weight"] = (dout, din, 1, 1)


def _linear_attention(p: str, dim: int, sd):
    # module_util.py:157-168 (heads=4, dim_head=32)
    sd[p + "to_qkv.weight"] = (384, dim, 1, 1)
    sd[p + "to_out.0.weight"] = (dim, 128, 1, 1)
    sd[p + "to_out.0.bias"] = (dim,)
    sd[p + "to_out.1.g"] = (1, dim, 1, 1)


def _spatial_transformer(p: str, dim: int, ctx: int, sd):
    # attention.py:218-248, BasicTransformerBlock 196-205, CrossAttention 152-168, GEGLU 37-44
    inner = dim  # n_heads * d_head = (dim // 32) * 32
    sd[p + "norm.weight"] = (dim,)
    sd[p + "norm.bias"] = (dim,)
    sd[p + "proj_in.weight"] = (inner, dim, 1, 1)
    sd[p + "proj_in.bias"] = (inner,)
    b = p + "transformer_blocks.0."
    sd[b + "attn1.to_q.weight"] = (inner, inner)
    sd[b + "attn1.to_k.weight"] = (inner, inner)
    sd[b + "attn1.to_v.weight"] = (inner, inner)
    sd[b + "attn1.to_out.0.weight"] = (inner, inner)
    sd[b + "attn1.to_out.0.bias"] = (inner,)
    sd[b + "ff.net.0.proj.weight"] = (inner * 8, inner)
    sd[b + "ff.net.0.proj.bias"] = (inner * 8,)
    sd[b + "ff.net.2.weight"] = (inner, inner * 4)
    sd[b + "ff.net.2.bias"] = (inner,)
    sd[b + "attn2.to_q.weight"] = (inner, inner)
    sd[b + "attn2.to_k.weight"] = (inner, ctx)
    sd[b + "attn2.to_v.weight"] = (inner, ctx)
    sd[b + "attn2.to_out.0.weight"] = (inner, inner)
    sd[b + "attn2.to_out.0.bias"] = (inner,)
    for n in ("norm1", "norm2", "norm3"):
        sd[b + n + ".weight"] = (inner,)
        sd[b + n + ".bias"] = (inner,)
    sd[p + "proj_out.weight"] = (dim, inner, 1, 1)
    sd[p + "proj_out.bias"] = (dim,)


def _attn(p: str, dim: int, use_st: bool, cfg: UNetConfig, sd):
    # Residual(PreNorm(dim, attn)): module_util.py:27-33, 89-97
    if use_st:
        _spatial_transformer(p + "fn.fn.", dim, cfg.context_dim, sd)
    else:
        _linear_attention(p + "fn.fn.", dim, sd)
    sd[p + "fn.norm.g"] = (1, dim, 1, 1)


def unet_state_spec(cfg: UNetConfig = UNetConfig()) -> "OrderedDict[str, Shape]":
    """Ordered {key: shape} identical to ConditionalUNet(**cfg).state_dict()."""
    sd: "OrderedDict[str, Shape]" = OrderedDict()
    nf, td = cfg.nf, cfg.time_dim
    if cfg.context_dim > 0 and cfg.use_degra_context:
        sd["prompt"] = (1, td)
    sd["init_conv.weight"] = (nf, cfg.in_nc * 2, 7, 7)
    if cfg.scale == 0.5:
        sd["downsample.weight"] = (nf, nf, 4, 4)
        sd["downsample.bias"] = (nf,)
        sd["upsample.1.weight"] = (nf, nf, 3, 3)
        sd["upsample.1.bias"] = (nf,)
    sd["time_mlp.1.weight"] = (td, nf)
    sd["time_mlp.1.bias"] = (td,)
    sd["time_mlp.3.weight"] = (td, td)
    sd["time_mlp.3.bias"] = (td,)
    if cfg.context_dim > 0 and cfg.use_degra_context:
        sd["text_mlp.0.weight"] = (td, cfg.context_dim)
        sd["text_mlp.0.bias"] = (td,)
        sd["text_mlp.2.weight"] = (td, td)
        sd["text_mlp.2.bias"] = (td,)
        sd["prompt_mlp.weight"] = (td, td)
        sd["prompt_mlp.bias"] = (td,)
    levels = cfg.levels()
    for i, (din, dout) in enumerate(levels):
        p = f"downs.{i}."
        _resblock(p + "0.", din, din, td, sd)
        _resblock(p + "1.", din, din, td, sd)
        _attn(p + "2.", din, cfg.uses_transformer(i), cfg, sd)
        if i != cfg.depth - 1:
            sd[p + "3.weight"] = (dout, din, 4, 4)
            sd[p + "3.bias"] = (dout,)
        else:
            sd[p + "3.weight"] = (dout, din, 3, 3)
    for j, i in enumerate(reversed(range(cfg.depth))):
        din, dout = levels[i]
        p = f"ups.{j}."
        _resblock(p + "0.", dout + din, dout, td, sd)
        _resblock(p + "1.", dout + din, dout, td, sd)
        _attn(p + "2.", dout, cfg.uses_transformer(i), cfg, sd)
        if i != 0:
            sd[p + "3.1.weight"] = (din, dout, 3, 3)
            sd[p + "3.1.bias"] = (din,)
        else:
            sd[p + "3.weight"] = (din, dout, 3, 3)
    mid = levels[-1][1]
    _resblock("mid_block1.", mid, mid, td, sd)
    _attn("mid_attn.", mid, cfg.use_image_context and cfg.context_dim > 0, cfg, sd)
    _resblock("mid_block2.", mid, mid, td, sd)
    _resblock("final_res_block.", nf * 2, nf, td, sd)
    sd["final_conv.weight"] = (cfg.out_nc, nf, 3, 3)
    sd["final_conv.bias"] = (cfg.out_nc,)
    return sd


# Wild-IR network_G.setting (config/wild-ir/options/inference.yml:30-39).
WILD_IR_UNET = UNetConfig(context_dim=768, use_degra_context=False, use_image_context=True,
                          scale=0.5, st_from=3)


# ----------------------------------------------------------------------------- DaCLIP

def _vit_tower(p: str, v: VisionConfig, sd, control: bool):
    w = v.width
    sd[p + "class_embedding"] = (w,)
    sd[p + "positional_embedding"] = (v.tokens, w)
    sd[p + "proj"] = (w, v.embed_dim)
    sd[p + "conv1.weight"] = (w, 3, v.patch_size, v.patch_size)
    sd[p + "ln_pre.weight"] = (w,)
    sd[p + "ln_pre.bias"] = (w,)
    rb = p + ("transformer.transformer.resblocks." if control else "transformer.resblocks.")
    hid = int(w * v.mlp_ratio)
    for l in range(v.layers):
        q = f"{rb}{l}."
        sd[q + "ln_1.weight"] = (w,)
        sd[q + "ln_1.bias"] = (w,)
        sd[q + "attn.in_proj_weight"] = (3 * w, w)
        sd[q + "attn.in_proj_bias"] = (3 * w,)
        sd[q + "attn.out_proj.weight"] = (w, w)
        sd[q + "attn.out_proj.bias"] = (w,)
        sd[q + "ln_2.weight"] = (w,)
        sd[q + "ln_2.bias"] = (w,)
        sd[q + "mlp.c_fc.weight"] = (hid, w)
        sd[q + "mlp.c_fc.bias"] = (hid,)
        sd[q + "mlp.c_proj.weight"] = (w, hid)
        sd[q + "mlp.c_proj.bias"] = (w,)
    if control:
        for l in range(v.layers):
            sd[f"{p}transformer.zero_modules.{l}.weight"] = (w, w)
            sd[f"{p}transformer.zero_modules.{l}.bias"] = (w,)
    sd[p + "ln_post.weight"] = (w,)
    sd[p + "ln_post.bias"] = (w,)


def _text_tower(t: TextConfig, embed_dim: int, sd):
    sd["clip.positional_embedding"] = (t.context_length, t.width)
    sd["clip.text_projection"] = (t.width, embed_dim)
    sd["clip.logit_scale"] = ()


def daclip_state_spec(vision: VisionConfig = VIT_B_32, text: TextConfig = TEXT_B_32
                      ) -> "OrderedDict[str, Shape]":
    """Ordered {key: shape} identical to DaCLIP(CLIP(**cfg)).state_dict() (631 keys for B/32)."""
    sd: "OrderedDict[str, Shape]" = OrderedDict()
    sd["logit_scale"] = ()
    _text_tower(text, vision.embed_dim, sd)
    _vit_tower("clip.visual.", vision, sd, control=False)
    w = text.width
    for l in range(text.layers):
        q = f"clip.transformer.resblocks.{l}."
        sd[q + "ln_1.weight"] = (w,)
        sd[q + "ln_1.bias"] = (w,)
        sd[q + "attn.in_proj_weight"] = (3 * w, w)
        sd[q + "attn.in_proj_bias"] = (3 * w,)
        sd[q + "attn.out_proj.weight"] = (w, w)
        sd[q + "attn.out_proj.bias"] = (w,)
        sd[q + "ln_2.weight"] = (w,)
        sd[q + "ln_2.bias"] = (w,)
        sd[q + "mlp.c_fc.weight"] = (4 * w, w)
        sd[q + "mlp.c_fc.bias"] = (4 * w,)
        sd[q + "mlp.c_proj.weight"] = (w, 4 * w)
        sd[q + "mlp.c_proj.bias"] = (w,)
    sd["clip.token_embedding.weight"] = (text.vocab_size, w)
    sd["clip.ln_final.weight"] = (w,)
    sd["clip.ln_final.bias"] = (w,)
    _vit_tower("visual.", vision, sd, control=False)
    _vit_tower("visual_control.", vision, sd, control=True)
    return sd


def canonical_daclip_key(k: str) -> str:
    """`visual.*` is an alias of `clip.visual.*` (daclip_model.py:21 shares the module)."""
    return "clip." + k if k.startswith("visual.") else k


def vision_keys(prefix: str, v: VisionConfig, control: bool) -> List[str]:
    sd: "OrderedDict[str, Shape]" = OrderedDict()
    _vit_tower(prefix, v, sd, control)
    return list(sd)


# ----------------------------------------------------------------------------- reference FLOPs
# The work the REFERENCE defines per forward, counted as torch.utils.flop_counter does on the
# reference's CPU path: 2*MAC over conv2d (2 x out elements x Cin x kh x kw),
# addmm / mm / bmm / einsum; nothing for norms, softmax, activations or elementwise ops, and —
# on the CPU path — nothing for the ViT's nn.MultiheadAttention core, which runs as the CPU
# flash SDPA kernel the counter has no formula for. These reproduce §8(d)'s constants from the
# shapes alone: 266.172 GF per UNet step at 256^2 (1129.09 at 512^2, Wild-IR 348.88 at 512^2),
# 18.159 GF per ViT-B/32 encode_image(control=True) (324.0 for ViT-L/14): 26.635 TF per
# restored 256^2 image at T = 100. The engine's own count (dac_unet_flops / dac_encode_flops)
# is the EXECUTED work, lower by the exact shortcuts it takes (one-key attn2 collapse, the
# LinearAttention re-association, row-phase upsample convs) and higher by the ViT attention.

def _conv(h: int, w: int, cin: int, cout: int, k: int) -> float:
    return 2.0 * h * w * cout * cin * k * k


def _ref_resblock(h, w, din, dout, td):
    # module_util.py:132-153: mlp Linear(td, 2 dout) on [1, td], two 3x3 convs, 1x1 res_conv
    f = 2.0 * td * 2 * dout + _conv(h, w, din, dout, 3) + _conv(h, w, dout, dout, 3)
    return f + (_conv(h, w, din, dout, 1) if din != dout else 0.0)


def _ref_linear_attention(h, w, c):
    # module_util.py:157-185: to_qkv 1x1 (c -> 384), two einsums over 4 heads x 32 x 32 x n,
    # to_out 1x1 (128 -> c)
    n = h * w
    return _conv(h, w, c, 384, 1) + 2 * (2.0 * 4 * 32 * 32 * n) + _conv(h, w, 128, c, 1)


def _ref_spatial_transformer(h, w, c, ctx):
    # attention.py:152-261 with one context token: proj_in / proj_out 1x1; attn1 q, k, v (mm),
    # q k^T and attn v (bmm, L^2 C each), to_out (addmm); attn2 to_q (mm), to_k / to_v on the
    # single context row, q k^T over that one key (a bmm of 2 L C; the attn x v einsum contracts
    # over j = 1, which torch.einsum evaluates as a broadcast multiply, not a bmm), to_out;
    # GEGLU proj (C -> 8C) and ff out (4C -> C)
    L = h * w
    f = 2 * _conv(h, w, c, c, 1)
    f += 3 * 2.0 * L * c * c + 2 * 2.0 * L * L * c + 2.0 * L * c * c
    f += 2.0 * L * c * c + 2 * 2.0 * ctx * c + 2.0 * L * c + 2.0 * L * c * c
    f += 2.0 * L * c * 8 * c + 2.0 * L * 4 * c * c
    return f


def reference_unet_flops(cfg: UNetConfig, H: int, W: int) -> float:
    """FLOPs of one ConditionalUNet.forward on one image (DenoisingUNet_arch.py:118-174; the
    Wild-IR variant's scale-0.5 down / up convs, config/wild-ir/.../DenoisingUNet_arch.py)."""
    s = 2 ** cfg.depth
    H, W = H + (s - H % s) % s, W + (s - W % s) % s           # check_image_size (reflect pad)
    nf, td = cfg.nf, cfg.time_dim
    f = _conv(H, W, 2 * cfg.in_nc, nf, 7)
    h, w = H, W
    if cfg.scale == 0.5:
        h, w = H // 2, W // 2
        f += _conv(h, w, nf, nf, 4)
    f += 2.0 * nf * td + 2.0 * td * td                         # time_mlp on the [1] time tensor
    if cfg.context_dim > 0 and cfg.use_degra_context:
        f += 2.0 * cfg.context_dim * td + 2.0 * td * td + 2.0 * td * td
    attn = lambda hh, ww, c, lvl: (_ref_spatial_transformer(hh, ww, c, cfg.context_dim)
                                   if cfg.uses_transformer(lvl) else _ref_linear_attention(hh, ww, c))
    levels = cfg.levels()
    for i, (din, dout) in enumerate(levels):
        f += 2 * _ref_resblock(h, w, din, din, td) + attn(h, w, din, i)
        if i != cfg.depth - 1:
            f += _conv(h // 2, w // 2, din, dout, 4)
            h, w = h // 2, w // 2
        else:
            f += _conv(h, w, din, dout, 3)
    mid = levels[-1][1]
    f += 2 * _ref_resblock(h, w, mid, mid, td)
    f += (_ref_spatial_transformer(h, w, mid, cfg.context_dim) if cfg.use_image_context and cfg.context_dim > 0
          else _ref_linear_attention(h, w, mid))
    for i in reversed(range(cfg.depth)):
        din, dout = levels[i]
        f += 2 * _ref_resblock(h, w, dout + din, dout, td) + attn(h, w, dout, i)
        if i != 0:
            h, w = 2 * h, 2 * w
        f += _conv(h, w, dout, din, 3)
    if cfg.scale == 0.5:
        h, w = 2 * h, 2 * w
        f += _conv(h, w, nf, nf, 3)
    f += _ref_resblock(h, w, 2 * nf, nf, td) + _conv(h, w, nf, cfg.out_nc, 3)
    return f


def reference_encode_flops(v: VisionConfig = VIT_B_32) -> float:
    """FLOPs of DaCLIP.encode_image(image, control=True) on one image (daclip_model.py:46-53):
    the controller tower (+ its 12 / 24 zero-module linears) and the CLIP tower, each a patch conv,
    `layers` ResidualAttentionBlocks (in_proj, out_proj, MLP) and the head projection."""
    L, wd = v.tokens, v.width
    hid = int(wd * v.mlp_ratio)
    tower = _conv(v.grid, v.grid, 3, wd, v.patch_size)
    tower += v.layers * (2.0 * L * wd * 3 * wd + 2.0 * L * wd * wd + 2 * 2.0 * L * wd * hid)
    tower += 2.0 * wd * v.embed_dim
    return 2 * tower + v.layers * 2.0 * L * wd * wd


def reference_tflop_per_image(cfg: UNetConfig, vision: VisionConfig, H: int, W: int, T: int) -> float:
    """T x F_unet(H, W) + F_clip, in TFLOP per restored image."""
    return (T * reference_unet_flops(cfg, H, W) + reference_encode_flops(vision)) / 1e12
