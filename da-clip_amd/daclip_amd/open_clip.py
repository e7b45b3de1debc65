"""open_clip mirror for the DA-CLIP image path, backed by libdaclip_hip.

Mirrors open_clip/factory.py:88-106 (load_state_dict / load_checkpoint key handling),
:109-269 (create_model, daclip branch 190-192, local-path checkpoint 231-241),
:365-404 (create_model_from_pretrained), daclip_model.py:46-55 (encode_image) and :125-126
(encode_text -> model.py:237-249), plus the degradation-class scoring of
da-clip/src/evaluate_daclip.py:45-50, 78-84.
"""
from __future__ import annotations

import os
import warnings
from typing import Mapping, Optional

import numpy as np
import torch

from . import _lib, arch, synth
from .preprocess import image_transform


def load_state_dict(checkpoint_path: str, map_location="cpu"):
    """factory.py:88-96: unwrap {'state_dict': ...} and strip a leading 'module.'."""
    ckpt = torch.load(checkpoint_path, map_location=map_location, weights_only=True)
    sd = ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt
    if next(iter(sd.items()))[0].startswith("module"):
        sd = {k[7:]: v for k, v in sd.items()}
    return sd


def vision_config(v: arch.VisionConfig, t: Optional[arch.TextConfig] = None) -> _lib.DacConfig:
    c = _lib.DacConfig()
    c.vit = 1
    c.image_size, c.patch_size, c.width = v.image_size, v.patch_size, v.width
    c.layers, c.head_width = v.layers, v.head_width
    c.mlp_width = int(v.width * v.mlp_ratio)
    c.embed_dim = v.embed_dim
    if t is not None:
        c.text = 1
        c.context_length, c.vocab_size = t.context_length, t.vocab_size
        c.text_width, c.text_heads, c.text_layers = t.width, t.heads, t.layers
    return c


def _is_text_key(k: str) -> bool:
    return k.startswith(("clip.transformer.", "clip.token_embedding.", "clip.ln_final.",
                         "clip.positional_embedding", "clip.text_projection"))


class DaCLIP:
    """DaCLIP(CLIP) image side: frozen clip.visual + controller visual_control."""

    def __init__(self, vision: arch.VisionConfig = arch.VIT_B_32,
                 text: arch.TextConfig = arch.TEXT_B_32, device="cuda", dtype="fp32",
                 with_text: bool = True):
        self.vision, self.text = vision, text
        self.with_text = with_text
        self._h = _lib.Handle(torch.device(device), dtype, vision_config(vision, text if with_text else None))
        self.device = self._h.device
        self.dtype = dtype
        self.visual = self          # exposes .image_size like VisionTransformer
        self.image_size = (vision.image_size, vision.image_size)
        self._loaded = False

    def state_spec(self):
        return arch.daclip_state_spec(self.vision, self.text)

    def load_state_dict(self, state_dict: Mapping[str, object], strict: bool = True):
        """Strict like factory.py:105. Deviation (documented): the training fork's extra
        `predictor.*` keys (da-clip/src/open_clip/daclip_model.py:92) are ignored with a
        warning instead of failing the strict load."""
        extra = [k for k in state_dict if k.startswith("predictor.")]
        if extra:
            warnings.warn(f"ignoring {len(extra)} predictor.* keys (training-only head)")
        spec = self.state_spec()
        keys = [k for k in state_dict if not k.startswith("predictor.")]
        missing = sorted(set(spec) - set(keys))
        # visual.* and clip.visual.* alias one module: either spelling satisfies the other.
        missing = [k for k in missing
                   if not (k.startswith("visual.") and "clip." + k in state_dict)
                   and not (k.startswith("clip.visual.") and k[5:] in state_dict)]
        unexpected = sorted(set(keys) - set(spec))
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for DaCLIP: missing keys {missing}, "
                               f"unexpected keys {unexpected}")
        for k in keys:
            if k not in spec:
                continue
            if k.startswith("visual.") and ("clip." + k) in state_dict:
                continue      # alias of clip.visual.* (same tensor)
            if not (k.startswith("clip.visual.") or k.startswith("visual") or
                    (self.with_text and _is_text_key(k))):
                continue      # logit scales (and the text tower when built without it)
            v = state_dict[k]
            t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
            if tuple(t.shape) != tuple(spec[k]):
                raise RuntimeError(f"size mismatch for {k}: {tuple(t.shape)} vs {spec[k]}")
            self._h.set_weight(k, t)
        self._h.finalize()
        self._loaded = True
        return missing, unexpected

    def load_synthetic(self, seed: int = 0):
        spec = {k: s for k, s in self.state_spec().items()
                if "visual" in k or (self.with_text and _is_text_key(k))}
        self.load_state_dict(synth.synth_state_dict(spec, seed), strict=False)

    def to(self, *a, **k):
        return self

    def eval(self):
        return self

    def encode_image(self, image: torch.Tensor, control: bool = False, normalize: bool = False):
        """daclip_model.py:46-55. control=True -> (image_features, degra_features), the
        controller's hiddens injected into the clip tower; control=False (the reference's
        default) -> CLIP.encode_image (model.py:233-235): the clip tower's features alone.
        [B, embed_dim] fp32."""
        if not self._loaded:
            raise RuntimeError("DaCLIP: weights not loaded")
        img = image.to(self.device, torch.float32).contiguous()
        B = img.shape[0]
        s = self.vision.image_size
        if tuple(img.shape[1:]) != (3, s, s):
            raise RuntimeError(f"expected [B,3,{s},{s}], got {tuple(img.shape)}")
        ic = torch.empty((B, self.vision.embed_dim), device=self.device, dtype=torch.float32)
        dc = torch.empty_like(ic) if control else None
        h = self._h
        with torch.cuda.device(self.device):
            h.check(_lib.lib().dac_encode_image(h.h, _lib._ptr(img), B, _lib._ptr(ic), _lib._ptr(dc),
                                                h.stream()), "encode_image")
        if not control:
            return torch.nn.functional.normalize(ic, dim=-1) if normalize else ic
        if normalize:
            ic = torch.nn.functional.normalize(ic, dim=-1)
            dc = torch.nn.functional.normalize(dc, dim=-1)
        return ic, dc

    def encode_text(self, text: torch.Tensor, normalize: bool = False) -> torch.Tensor:
        """daclip_model.py:125-126 -> CLIP.encode_text (model.py:237-249): token ids
        [N, context_length] (open_clip.tokenize output) -> [N, embed_dim] fp32."""
        if not self.with_text:
            raise RuntimeError("DaCLIP built with with_text=False")
        if not self._loaded:
            raise RuntimeError("DaCLIP: weights not loaded")
        tok = text.to(self.device, torch.int64).contiguous()
        if tok.dim() != 2 or tok.shape[1] != self.text.context_length:
            raise RuntimeError(f"expected [N,{self.text.context_length}] token ids, got {tuple(tok.shape)}")
        out = torch.empty((tok.shape[0], self.vision.embed_dim), device=self.device, dtype=torch.float32)
        h = self._h
        with torch.cuda.device(self.device):
            h.check(_lib.lib().dac_encode_text(h.h, _lib._ptr(tok), tok.shape[0], _lib._ptr(out), h.stream()),
                    "encode_text")
        return torch.nn.functional.normalize(out, dim=-1) if normalize else out

    def degradation_probs(self, degra_features: torch.Tensor, text_features: torch.Tensor):
        """evaluate_daclip.py:45-50, 78-84: probs = softmax(100 * d^ t^T) over the K class
        texts and argmax (first maximum) -> (probs [B, K] fp32, argmax [B] int64)."""
        d = degra_features.to(self.device, torch.float32).contiguous()
        t = text_features.to(self.device, torch.float32).contiguous()
        B, E = d.shape
        K = t.shape[0]
        probs = torch.empty((B, K), device=self.device, dtype=torch.float32)
        am = torch.empty((B,), device=self.device, dtype=torch.int32)
        h = self._h
        with torch.cuda.device(self.device):
            h.check(_lib.lib().dac_degradation_probs(h.h, _lib._ptr(d), _lib._ptr(t), B, K, E, _lib._ptr(probs),
                                                     _lib._ptr(am), h.stream()), "degradation_probs")
        return probs, am.long()

    def flops(self, B: int) -> float:
        return _lib.lib().dac_encode_flops(self._h.h, B)


def create_model(model_name: str, pretrained: Optional[str] = None, precision: str = "fp32",
                 device="cuda", require_pretrained: bool = False, dtype: Optional[str] = None,
                 **_):
    if model_name not in arch.MODEL_CONFIGS:
        raise RuntimeError(f"Model config for {model_name} not found.")
    v, t = arch.MODEL_CONFIGS[model_name]
    # factory.py:198-219: 'fp16'/'bf16' (manual mixed precision) and 'pure_fp16'/'pure_bf16'
    # store the weights in 16 bits; 'amp' / 'amp_bf16' keep fp32 weights (autocast is the
    # caller's business there), so they map to the fp32 handles here too.
    dt = dtype or ("bf16" if precision in ("bf16", "pure_bf16") else
                   "fp16" if precision in ("fp16", "pure_fp16") else "fp32")
    model = DaCLIP(v, t, device=device, dtype=dt)
    if pretrained:
        if not os.path.exists(pretrained):
            raise RuntimeError(f"Pretrained weights ({pretrained}) not found for model {model_name}.")
        model.load_state_dict(load_state_dict(pretrained), strict=True)
    elif require_pretrained:
        raise RuntimeError(f"Pretrained weights were required for (model: {model_name}) but not loaded.")
    return model


def create_model_from_pretrained(model_name: str, pretrained: Optional[str] = None,
                                 precision: str = "fp32", device="cuda",
                                 return_transform: bool = True, dtype: Optional[str] = None, **kw):
    model = create_model(model_name, pretrained, precision, device, require_pretrained=True,
                         dtype=dtype)
    if not return_transform:
        return model
    return model, image_transform(model.vision.image_size)
