"""ConditionalUNet mirror (DenoisingUNet_arch.py:22-174) backed by libdaclip_hip.

`ConditionalUNet(**network_G.setting)` has the reference constructor signature; the module is
callable as `model(xt, cond, time, text_context=None, image_context=None) -> noise`, i.e. it
is a drop-in for the `sde.set_model(...)` plug point (sde_utils.py:163-164, 195-202).
Weights enter through `load_state_dict` (strict, like base_model.py:92-105 load_network).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Mapping, Optional, Sequence

import numpy as np
import torch

from . import _lib, arch, synth


def unet_config(cfg: arch.UNetConfig) -> _lib.DacConfig:
    c = _lib.DacConfig()
    c.unet = 1
    c.in_nc, c.out_nc, c.nf = cfg.in_nc, cfg.out_nc, cfg.nf
    c.depth = cfg.depth
    for i, m in enumerate(cfg.ch_mult):
        c.ch_mult[i] = m
    c.context_dim = cfg.context_dim if cfg.context_dim is not None else -1
    c.use_degra_context = int(cfg.use_degra_context)
    c.use_image_context = int(cfg.use_image_context)
    if cfg.scale not in (1, 0.5):
        raise ValueError(f"scale {cfg.scale}: only 1 and 0.5 exist in the reference")
    c.unet_scale_half = int(cfg.scale == 0.5)
    c.unet_st_from = cfg.st_from
    return c


def _incompatible(expected: Sequence[str], got: Sequence[str]):
    exp, g = set(expected), set(got)
    return sorted(exp - g), sorted(g - exp)


class ConditionalUNet:
    def __init__(self, in_nc=3, out_nc=3, nf=64, ch_mult=(1, 2, 4, 4), context_dim=512,
                 use_degra_context=True, use_image_context=False, upscale=1, scale=1,
                 device="cuda", dtype="fp32"):
        """daclip-sde signature (`upscale`, unused there) plus the Wild-IR `scale` (0.5 adds the
        half-resolution wrap, config/wild-ir/models/modules/DenoisingUNet_arch.py:22-40)."""
        depth = len(ch_mult)
        self.cfg = arch.UNetConfig(in_nc, out_nc, nf, tuple(ch_mult), context_dim,
                                   bool(use_degra_context), bool(use_image_context),
                                   scale=scale, st_from=depth - 1 if scale != 1 else 3)
        self.depth = self.cfg.depth
        self.upscale = upscale
        self.dtype = dtype
        self.device = torch.device(device)
        self._h = _lib.Handle(self.device, dtype, unet_config(self.cfg))
        self.device = self._h.device
        self._loaded = False

    # -------------------------------------------------------------- weights
    def state_spec(self):
        return arch.unet_state_spec(self.cfg)

    def load_state_dict(self, state_dict: Mapping[str, object], strict: bool = True):
        spec = self.state_spec()
        missing, unexpected = _incompatible(list(spec), list(state_dict))
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for ConditionalUNet: "
                               f"missing keys {missing}, unexpected keys {unexpected}")
        for k in spec:
            v = state_dict[k]
            t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
            if tuple(t.shape) != tuple(spec[k]):
                raise RuntimeError(f"size mismatch for {k}: copying a param with shape "
                                   f"{tuple(t.shape)}, the shape in current model is {spec[k]}")
            self._h.set_weight(k, t)
        self._h.finalize()
        self._loaded = True
        return missing, unexpected

    def load_synthetic(self, seed: int = 0):
        """Deterministic random-init weights (no checkpoint offline), see synth.py."""
        return self.load_state_dict(synth.synth_state_dict(self.state_spec(), seed))

    # -------------------------------------------------------------- compute
    def _prep(self, t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if t is None:
            return None
        return t.to(self.device, torch.float32).contiguous()

    def __call__(self, xt, cond, time, text_context=None, image_context=None):
        return self.forward(xt, cond, time, text_context, image_context)

    def forward(self, xt, cond, time, text_context=None, image_context=None):
        """DenoisingUNet_arch.py:118-174. `time` is a python number or a 1-element tensor."""
        if not self._loaded:
            raise RuntimeError("ConditionalUNet: load_state_dict() first")
        if isinstance(time, torch.Tensor):
            if time.numel() != 1:
                raise RuntimeError("per-sample timesteps are a training-path feature (out of scope)")
            time = float(time.reshape(-1)[0].item())
        xt, cond = self._prep(xt), self._prep(cond)
        tc = self._prep(text_context) if self.cfg.use_degra_context else None
        ic = self._prep(image_context) if self.cfg.use_image_context else None
        B, C, H, W = xt.shape
        out = torch.empty((B, self.cfg.out_nc, H, W), device=self.device, dtype=torch.float32)
        h = self._h
        with torch.cuda.device(self.device):
            h.check(_lib.lib().dac_unet_forward(h.h, _lib._ptr(xt), _lib._ptr(cond), float(time),
                                                _lib._ptr(tc), _lib._ptr(ic), B, H, W,
                                                _lib._ptr(out), h.stream()), "unet_forward")
        return out

    def eval(self):
        return self

    def train(self, mode=True):
        return self

    def flops(self, B: int, H: int, W: int) -> float:
        """Executed FLOPs (2*MAC) of one forward."""
        return _lib.lib().dac_unet_flops(self._h.h, B, H, W)
