"""numpy restatement of ConditionalUNet.forward (CPU oracle; TEST INFRASTRUCTURE ONLY).

Follows universal-image-restoration/config/daclip-sde/models/modules/
  DenoisingUNet_arch.py:118-174 (forward), module_util.py:27-185 (ResBlock, LinearAttention,
  LayerNorm, PreNorm, Up/Downsample, SinusoidalPosEmb), attention.py:37-261
  (GEGLU, CrossAttention, BasicTransformerBlock, SpatialTransformer).
`sd` is a {state_dict key: float32 ndarray} mapping with the reference's key names.
"""
from __future__ import annotations

import math

import numpy as np

from . import nn as F

f32 = np.float32


def sinusoidal_pos_emb(t, dim):
    """module_util.py:36-48."""
    half = dim // 2
    emb = math.log(10000) / (half - 1)
    emb = np.exp(np.arange(half, dtype=f32) * f32(-emb)).astype(f32)
    emb = np.asarray(t, f32).reshape(-1)[:, None] * emb[None, :]
    return np.concatenate([np.sin(emb), np.cos(emb)], -1).astype(f32)


def resblock(sd, p, x, temb):
    """module_util.py:132-153: SiLU(conv(x)*(s+1)+sh) -> SiLU(conv) -> + res_conv(x)."""
    ss = F.linear(F.silu(temb), sd[p + "mlp.1.weight"], sd[p + "mlp.1.bias"])
    c = ss.shape[1] // 2
    scale, shift = ss[:, :c, None, None], ss[:, c:, None, None]
    h = F.conv2d(x, sd[p + "block1.proj.weight"], pad=1)
    h = F.silu(h * (scale + 1) + shift)
    h = F.silu(F.conv2d(h, sd[p + "block2.proj.weight"], pad=1))
    res = F.conv2d(x, sd[p + "res_conv.weight"]) if (p + "res_conv.weight") in sd else x
    return (h + res).astype(f32)


def linear_attention(sd, p, x):
    """module_util.py:157-185 (heads=4, dim_head=32)."""
    b, c, h, w = x.shape
    qkv = F.conv2d(x, sd[p + "to_qkv.weight"])
    q, k, v = [t.reshape(b, 4, 32, h * w) for t in np.split(qkv, 3, axis=1)]
    q = F.softmax(q, axis=-2)
    k = F.softmax(k, axis=-1)
    q = q * f32(32 ** -0.5)
    v = v / f32(h * w)
    ctx = np.einsum("bhdn,bhen->bhde", k, v).astype(f32)
    out = np.einsum("bhde,bhdn->bhen", ctx, q).astype(f32).reshape(b, 128, h, w)
    out = F.conv2d(out, sd[p + "to_out.0.weight"], sd[p + "to_out.0.bias"])
    return F.channel_layer_norm(out, sd[p + "to_out.1.g"])


def cross_attention(sd, p, x, ctx, heads):
    """attention.py:170-193. x [B,N,C], ctx [B,M,Cc]."""
    q = F.linear(x, sd[p + "to_q.weight"])
    k = F.linear(ctx, sd[p + "to_k.weight"])
    v = F.linear(ctx, sd[p + "to_v.weight"])
    B, N, inner = q.shape
    d = inner // heads
    sp = lambda t: t.reshape(B, t.shape[1], heads, d).transpose(0, 2, 1, 3)
    q, k, v = sp(q), sp(k), sp(v)
    sim = (q @ k.transpose(0, 1, 3, 2)) * f32(d ** -0.5)
    out = (F.softmax(sim, -1) @ v).transpose(0, 2, 1, 3).reshape(B, N, inner)
    return F.linear(out, sd[p + "to_out.0.weight"], sd[p + "to_out.0.bias"])


def spatial_transformer(sd, p, x, ctx):
    """attention.py:250-261 with one BasicTransformerBlock (211-215), GEGLU FF (37-64)."""
    b, c, h, w = x.shape
    heads = c // 32
    x_in = x
    x = F.group_norm(x, 32, sd[p + "norm.weight"], sd[p + "norm.bias"], eps=1e-6)
    x = F.conv2d(x, sd[p + "proj_in.weight"], sd[p + "proj_in.bias"])
    x = x.reshape(b, c, h * w).transpose(0, 2, 1)
    q = p + "transformer_blocks.0."
    ln = lambda n, t: F.layer_norm(t, sd[q + n + ".weight"], sd[q + n + ".bias"])
    x = cross_attention(sd, q + "attn1.", ln("norm1", x), ln("norm1", x), heads) + x
    # attn2: cross-attention on the context, or self-attention when none is given (:174).
    xn2 = ln("norm2", x)
    x = cross_attention(sd, q + "attn2.", xn2, xn2 if ctx is None else ctx, heads) + x
    hdn = F.linear(ln("norm3", x), sd[q + "ff.net.0.proj.weight"], sd[q + "ff.net.0.proj.bias"])
    a, gate = np.split(hdn, 2, axis=-1)
    x = F.linear(a * F.gelu(gate), sd[q + "ff.net.2.weight"], sd[q + "ff.net.2.bias"]) + x
    x = x.transpose(0, 2, 1).reshape(b, c, h, w)
    x = F.conv2d(x, sd[p + "proj_out.weight"], sd[p + "proj_out.bias"])
    return (x + x_in).astype(f32)


def attn_block(sd, p, x, ctx):
    """Residual(PreNorm(dim, attn)) (module_util.py:27-33, 89-97)."""
    xn = F.channel_layer_norm(x, sd[p + "fn.norm.g"])
    if (p + "fn.fn.to_qkv.weight") in sd:
        y = linear_attention(sd, p + "fn.fn.", xn)
    else:
        y = spatial_transformer(sd, p + "fn.fn.", xn, ctx)
    return (y + x).astype(f32)


def time_embedding(sd, t, nf, text_context=None):
    """DenoisingUNet_arch.py:132-137: [1,T] time MLP (+ [B,T] prompt embedding)."""
    te = sinusoidal_pos_emb(t, nf)
    te = F.linear(te, sd["time_mlp.1.weight"], sd["time_mlp.1.bias"])
    te = F.linear(F.gelu(te), sd["time_mlp.3.weight"], sd["time_mlp.3.bias"])
    if text_context is not None and "text_mlp.0.weight" in sd:
        pe = F.linear(text_context, sd["text_mlp.0.weight"], sd["text_mlp.0.bias"])
        pe = F.linear(F.silu(pe), sd["text_mlp.2.weight"], sd["text_mlp.2.bias"])
        pe = F.softmax(pe, 1) * sd["prompt"]
        pe = F.linear(pe, sd["prompt_mlp.weight"], sd["prompt_mlp.bias"])
        te = (te + pe).astype(f32)
    return te


def forward(sd, xt, cond, time, text_context=None, image_context=None, depth=4):
    """ConditionalUNet.forward (DenoisingUNet_arch.py:118-174; the Wild-IR variant's half-scale
    wrap, config/wild-ir/models/modules/DenoisingUNet_arch.py:122-189, is keyed on its weights)."""
    nf = sd["init_conv.weight"].shape[0]
    x = np.concatenate([xt - cond, cond], 1).astype(f32)
    H, W = x.shape[2:]
    s = 2 ** depth
    x = F.reflect_pad(x, (s - H % s) % s, (s - W % s) % s)
    x = F.conv2d(x, sd["init_conv.weight"], pad=3)
    x_ = x.copy()
    if "downsample.weight" in sd:                # Wild-IR scale 0.5 (wild-ir arch :136-140)
        x = F.conv2d(x, sd["downsample.weight"], sd["downsample.bias"], stride=2, pad=1)
    t = time_embedding(sd, time, nf, text_context)
    ctx = image_context[:, None, :] if image_context is not None else None

    h = []
    for i in range(depth):
        p = f"downs.{i}."
        x = resblock(sd, p + "0.", x, t)
        h.append(x)
        x = resblock(sd, p + "1.", x, t)
        x = attn_block(sd, p + "2.", x, ctx)
        h.append(x)
        if i != depth - 1:
            x = F.conv2d(x, sd[p + "3.weight"], sd[p + "3.bias"], stride=2, pad=1)
        else:
            x = F.conv2d(x, sd[p + "3.weight"], pad=1)
    x = resblock(sd, "mid_block1.", x, t)
    x = attn_block(sd, "mid_attn.", x, ctx)
    x = resblock(sd, "mid_block2.", x, t)
    for j in range(depth):
        p = f"ups.{j}."
        x = np.concatenate([x, h.pop()], 1)
        x = resblock(sd, p + "0.", x, t)
        x = np.concatenate([x, h.pop()], 1)
        x = resblock(sd, p + "1.", x, t)
        x = attn_block(sd, p + "2.", x, ctx)
        if (p + "3.1.weight") in sd:
            x = F.conv2d(F.upsample_nearest2x(x), sd[p + "3.1.weight"], sd[p + "3.1.bias"], pad=1)
        else:
            x = F.conv2d(x, sd[p + "3.weight"], pad=1)
    if "upsample.1.weight" in sd:                # wild-ir arch :176-180
        x = F.conv2d(F.upsample_nearest2x(x), sd["upsample.1.weight"], sd["upsample.1.bias"], pad=1)
    x = np.concatenate([x, x_], 1)
    x = resblock(sd, "final_res_block.", x, t)
    x = F.conv2d(x, sd["final_conv.weight"], sd["final_conv.bias"], pad=1)
    return np.ascontiguousarray(x[..., :H, :W])
