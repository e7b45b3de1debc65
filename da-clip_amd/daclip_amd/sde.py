"""IRSDE mirror (utils/sde_utils.py:80-378), inference part.

The schedule tables are computed with the same torch fp32 CPU ops as the reference
(_initialize, sde_utils.py:91-154), so they are bit-identical to it, and handed to the native
library. `reverse_posterior` / `reverse_sde` with a native ConditionalUNet run the whole
T-step loop inside libdaclip_hip as one captured hipGraph (dac_sde_reverse); with any other
callable model they run the reference's Python loop, with the sampler update itself still a
library kernel (dac_posterior_step).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _lib
from .preprocess import save_image
from .unet import ConditionalUNet


class IRSDE:
    """Let timestep t start from 1 to T, state t=0 is never used (sde_utils.py:80-83)."""

    def __init__(self, max_sigma, T=100, sample_T=-1, schedule="cosine", eps=0.01, device=None):
        self.T = T
        self.dt = 1 / T
        self.device = device
        self.max_sigma = max_sigma / 255 if max_sigma >= 1 else max_sigma
        self.sample_T = self.T if sample_T < 0 else sample_T
        self.sample_scale = self.T / self.sample_T
        self.schedule = schedule
        self.eps = eps
        self._initialize(self.max_sigma, self.sample_T, schedule, eps)
        self.seed = 0
        # Global index of image 0 of the batch this process restores (sharded runs): the
        # device noise of image b is keyed by image_offset + b (dac_set_noise_offset).
        self.image_offset = 0

    def _initialize(self, max_sigma, T, schedule, eps=0.01):
        # Verbatim torch op sequence of sde_utils.py:112-151 (fp32 CPU).
        if schedule == "cosine":
            timesteps = T + 2
            steps = timesteps + 1
            x = torch.linspace(0, timesteps, steps, dtype=torch.float32)
            ac = torch.cos(((x / timesteps) + 0.008) / (1 + 0.008) * math.pi * 0.5) ** 2
            ac = ac / ac[0]
            thetas = 1 - ac[1:-1]
        elif schedule == "linear":
            timesteps = T + 1
            scale = 1000 / timesteps
            thetas = torch.linspace(scale * 0.0001, scale * 0.02, timesteps, dtype=torch.float32)
        elif schedule == "constant":
            thetas = torch.ones(T + 1, dtype=torch.float32)
        else:
            raise ValueError(f"unknown schedule {schedule}")
        sigmas = torch.sqrt(max_sigma ** 2 * 2 * thetas)
        thetas_cumsum = torch.cumsum(thetas, dim=0) - thetas[0]
        self.dt = -1 / thetas_cumsum[-1] * math.log(eps)
        sigma_bars = torch.sqrt(max_sigma ** 2 * (1 - torch.exp(-2 * thetas_cumsum * self.dt)))
        self.thetas, self.sigmas = thetas, sigmas
        self.thetas_cumsum, self.sigma_bars = thetas_cumsum, sigma_bars
        self.mu = 0.0
        self.model = None

    def _tables(self) -> torch.Tensor:
        return torch.cat([self.thetas, self.sigmas, self.thetas_cumsum, self.sigma_bars]).float()

    def _sync_schedule(self, h: _lib.Handle):
        sched = {"cosine": _lib.DAC_COSINE, "linear": _lib.DAC_LINEAR,
                 "constant": _lib.DAC_CONSTANT}[self.schedule]
        tab = self._tables().contiguous()
        h.check(_lib.lib().dac_sde_schedule(h.h, float(self.max_sigma), int(self.sample_T), sched,
                                            float(self.eps), _lib.ctypes.c_void_p(tab.data_ptr()),
                                            float(self.dt)), "sde_schedule")

    # ------------------------------------------------------------------ plug points
    def set_mu(self, mu):
        self.mu = mu

    def set_model(self, model):
        self.model = model

    def noise_state(self, tensor, noise: Optional[torch.Tensor] = None):
        """sde_utils.py:374-375. `noise` may be injected (parity tests)."""
        z = torch.randn_like(tensor) if noise is None else noise.to(tensor)
        return tensor + z * self.max_sigma

    # ------------------------------------------------------------------ reference math
    def sigma_bar(self, t):
        return self.sigma_bars[t]

    def get_score_from_noise(self, noise, t):
        return -noise / self.sigma_bar(t)

    def noise_fn(self, x, t, scale=1.0, **kwargs):
        return self.model(x, self.mu, t * scale, **kwargs)

    def score_fn(self, x, t, scale=1.0, **kwargs):
        return self.get_score_from_noise(self.noise_fn(x, t, scale, **kwargs), t)

    # ------------------------------------------------------------------ samplers
    def _native(self):
        return self.model if isinstance(self.model, ConditionalUNet) else None

    def _save_state(self, x, t, save_dir):
        """sde_utils.py:269-275 / 305-311 verbatim semantics: every T // 100 steps (T < 100 makes
        the interval 0 and raises, as in the reference), channel halves side by side (an odd
        channel count fails in torch.cat exactly like the reference), save_image PNG."""
        interval = self.T // 100
        if t % interval == 0:
            idx = t // interval
            os.makedirs(save_dir, exist_ok=True)
            x_l, x_r = x.detach().cpu().chunk(2, dim=1)
            save_image(torch.cat([x_l, x_r], dim=3), f"{save_dir}/state_{idx}.png")

    def _loop(self, mode, xt, T, noises, save_states=False, save_dir="state", **kwargs):
        m = self._native()
        mu = self.mu if isinstance(self.mu, torch.Tensor) else torch.full_like(xt, float(self.mu))
        if m is not None and not save_states:
            h = m._h
            dev = m.device
            x = xt.to(dev, torch.float32).contiguous().clone()
            mu_d = mu.to(dev, torch.float32).contiguous()
            tc = kwargs.get("text_context")
            ic = kwargs.get("image_context")
            tc = tc.to(dev, torch.float32).contiguous() if (tc is not None and m.cfg.use_degra_context) else None
            ic = ic.to(dev, torch.float32).contiguous() if (ic is not None and m.cfg.use_image_context) else None
            nz = None
            if noises is not None:
                nz = noises[:T].to(dev, torch.float32).contiguous()
            B, _, H, W = x.shape
            with torch.cuda.device(dev):
                self._sync_schedule(h)
                # the model sees t * sample_scale (sde_utils.py:266, 302)
                h.check(_lib.lib().dac_sde_set_time_scale(h.h, float(self.sample_scale)), "time_scale")
                self.seed += 1
                h.check(_lib.lib().dac_set_noise_offset(h.h, int(self.image_offset)), "noise_offset")
                h.check(_lib.lib().dac_sde_reverse(h.h, mode, _lib._ptr(x), _lib._ptr(mu_d),
                                                   _lib._ptr(tc), _lib._ptr(ic), B, H, W, int(T),
                                                   _lib._ptr(nz), self.seed, h.stream()),
                        "sde_reverse")
            return x
        # Generic callable model (or save_states): the reference's per-step loop
        # (sde_utils.py:297-313 / 261-277) with the native sampler update.
        x = xt.clone().float()
        for i, t in enumerate(range(T, 0, -1)):
            eps = self.noise_fn(x, t, self.sample_scale, **kwargs).float().contiguous()
            z = noises[i] if noises is not None else torch.randn_like(x)
            x = self.step(mode, x, eps, mu, z, t)
            if save_states:
                self._save_state(x, t, save_dir)
        return x

    def step(self, mode, x, eps, mu, z, t):
        """One native sampler update (reverse_posterior_step / reverse_sde_step)."""
        h = getattr(self, "_step_handle", None)
        dev = x.device
        if h is None or h.device != dev:
            h = _lib.Handle(dev, "fp32", _lib.DacConfig())
            self._step_handle = h
        self._sync_schedule(h)
        for name, v in (("eps", eps), ("mu", mu), ("z", z)):
            if v.numel() != x.numel():
                raise RuntimeError(f"step: {name} has {v.numel()} elements, x has {x.numel()}")
        out = x.contiguous().clone()
        with torch.cuda.device(dev):
            h.check(_lib.lib().dac_posterior_step(h.h, mode, _lib._ptr(out), _lib._ptr(eps.contiguous()),
                                                  _lib._ptr(mu.to(dev).float().contiguous()),
                                                  _lib._ptr(z.to(dev).float().contiguous()), int(t),
                                                  out.numel(), h.stream()), "posterior_step")
        return out

    def reverse_posterior(self, xt, T=-1, save_states=False, save_dir="posterior_state",
                          noises=None, **kwargs):
        T = self.sample_T if T < 0 else T
        return self._loop(_lib.DAC_POSTERIOR, xt, T, noises, save_states, save_dir, **kwargs)

    def reverse_sde(self, xt, T=-1, save_states=False, save_dir="sde_state", noises=None, **kwargs):
        T = self.sample_T if T < 0 else T
        return self._loop(_lib.DAC_SDE, xt, T, noises, save_states, save_dir, **kwargs)
