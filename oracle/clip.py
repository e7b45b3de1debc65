"""numpy restatement of DaCLIP.encode_image(control=True) (CPU oracle; TEST INFRASTRUCTURE ONLY).

Follows open_clip/daclip_model.py:46-53, open_clip/transformer.py:189-244
(ResidualAttentionBlock with nn.MultiheadAttention), 288-325 (ControlTransformer),
355-369 (Transformer.forward with `x += control.pop()`), 507-555 (VisionTransformer.forward).
Tokens are kept batch-major [B, L, D]; the reference's LND permute is a pure relayout.
"""
from __future__ import annotations

import numpy as np

from . import nn as F

f32 = np.float32


def mha(x, w_in, b_in, w_out, b_out, heads, causal=False):
    """nn.MultiheadAttention(q=k=v=x), need_weights=False; optional additive causal mask
    (-inf above the diagonal, transformer.py:751-757). x [B,L,D]."""
    B, L, D = x.shape
    d = D // heads
    qkv = F.linear(x, w_in, b_in)
    q, k, v = [t.reshape(B, L, heads, d).transpose(0, 2, 1, 3) for t in np.split(qkv, 3, -1)]
    s = (q * f32(d ** -0.5)) @ k.transpose(0, 1, 3, 2)
    if causal:
        s = s + np.triu(np.full((L, L), -np.inf, f32), 1)
    o = (F.softmax(s, -1) @ v).transpose(0, 2, 1, 3).reshape(B, L, D)
    return F.linear(o, w_out, b_out)


def resblock(sd, p, x, heads, causal=False):
    """ResidualAttentionBlock.forward (transformer.py:232-244), ls_* = Identity."""
    h = F.layer_norm(x, sd[p + "ln_1.weight"], sd[p + "ln_1.bias"])
    x = x + mha(h, sd[p + "attn.in_proj_weight"], sd[p + "attn.in_proj_bias"],
                sd[p + "attn.out_proj.weight"], sd[p + "attn.out_proj.bias"], heads, causal)
    h = F.layer_norm(x, sd[p + "ln_2.weight"], sd[p + "ln_2.bias"])
    h = F.gelu(F.linear(h, sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"]))
    return (x + F.linear(h, sd[p + "mlp.c_proj.weight"], sd[p + "mlp.c_proj.bias"])).astype(f32)


def vision_forward(sd, p, img, layers, heads, control_tower=False, control=None):
    """VisionTransformer.forward (transformer.py:507-555) on NCHW img."""
    w = sd[p + "conv1.weight"]
    ps = w.shape[-1]
    x = F.conv2d(img, w, stride=ps)                      # [B, D, g, g]
    B, D = x.shape[:2]
    x = x.reshape(B, D, -1).transpose(0, 2, 1)           # [B, g*g, D]
    cls = np.broadcast_to(sd[p + "class_embedding"], (B, 1, D))
    x = np.concatenate([cls, x], 1) + sd[p + "positional_embedding"]
    x = F.layer_norm(x, sd[p + "ln_pre.weight"], sd[p + "ln_pre.bias"]).astype(f32)
    rb = p + ("transformer.transformer.resblocks." if control_tower else "transformer.resblocks.")
    hiddens = []
    control = list(control) if control is not None else None
    for l in range(layers):
        x = resblock(sd, f"{rb}{l}.", x, heads)
        if control_tower:
            hiddens.append(F.linear(x, sd[f"{p}transformer.zero_modules.{l}.weight"],
                                    sd[f"{p}transformer.zero_modules.{l}.bias"]))
        if control is not None:
            x = (x + control.pop()).astype(f32)         # transformer.py:367-368 (LIFO)
    pooled = F.layer_norm(x[:, 0], sd[p + "ln_post.weight"], sd[p + "ln_post.bias"])
    pooled = (pooled @ sd[p + "proj"]).astype(f32)
    return (pooled, hiddens) if control_tower else pooled


def encode_image(sd, img, layers=None, heads=None, control=True):
    """DaCLIP.encode_image(image, control=True) -> (image_features, degra_features)
    (daclip_model.py:46-53); control=False -> CLIP.encode_image (daclip_model.py:54-55,
    model.py:233-235): the clip tower's features alone."""
    width = sd["clip.visual.class_embedding"].shape[0]
    heads = heads or width // 64
    if layers is None:
        layers = 1 + max(int(k.split(".")[4]) for k in sd
                         if k.startswith("clip.visual.transformer.resblocks."))
    if not control:
        return vision_forward(sd, "clip.visual.", img, layers, heads)
    degra, hiddens = vision_forward(sd, "visual_control.", img, layers, heads, control_tower=True)
    image = vision_forward(sd, "clip.visual.", img, layers, heads, control=hiddens)
    return image, degra


def encode_text(sd, tokens, heads=8):
    """CLIP.encode_text (model.py:237-249; DaCLIP.encode_text daclip_model.py:125-126):
    token + positional embedding, causal ResidualAttentionBlocks, ln_final, the EOT token's
    features (position of the highest id, model.py:248) @ text_projection. tokens [N, L] int."""
    p = "clip."
    tokens = np.asarray(tokens)
    x = sd[p + "token_embedding.weight"][tokens] + sd[p + "positional_embedding"][None]
    layers = len({k.split(".")[3] for k in sd if k.startswith(p + "transformer.resblocks.")})
    for l in range(layers):
        x = resblock(sd, f"{p}transformer.resblocks.{l}.", x.astype(f32), heads, causal=True)
    x = F.layer_norm(x, sd[p + "ln_final.weight"], sd[p + "ln_final.bias"])
    pooled = x[np.arange(x.shape[0]), tokens.argmax(-1)]
    return (pooled @ sd[p + "text_projection"]).astype(f32)


def degradation_probs(degra, text_features):
    """evaluate_daclip.py:45-50, 78-84: softmax(100 * d^ t^T) over the class texts."""
    d = degra / np.linalg.norm(degra, axis=-1, keepdims=True)
    t = text_features / np.linalg.norm(text_features, axis=-1, keepdims=True)
    return F.softmax(f32(100.0) * (d @ t.T), -1).astype(f32)

