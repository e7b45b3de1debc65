"""numpy restatement of IRSDE (CPU oracle; TEST INFRASTRUCTURE ONLY).

Follows universal-image-restoration/utils/sde_utils.py:84-154 (_initialize: cosine/linear
theta schedules, sigmas, thetas_cumsum, dt, sigma_bars), 177-231 (reverse drift, dispersion,
reverse_optimum_step/std, reverse_posterior_step), 245-247 (get_init_state_from_noise),
261-313 (reverse_sde / reverse_posterior loops) and 374-375 (noise_state). Random draws are
injected (noise arrays) instead of torch.randn_like, matching tests/golden/make_golden.py.
Scalar table math is float32, like the reference's 0-dim torch tensors.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


class IRSDE:
    def __init__(self, max_sigma=50, T=100, schedule="cosine", eps=0.005, sample_T=-1):
        # sde_utils.py:84-89: the schedule is built over sample_T steps and the model is called
        # at t * sample_scale, sample_scale = T / sample_T.
        self.sample_scale = T / sample_T if sample_T > 0 else 1.0
        T = sample_T if sample_T > 0 else T
        self.T = T
        self.max_sigma = max_sigma / 255 if max_sigma >= 1 else max_sigma
        ms = self.max_sigma
        if schedule == "cosine":                   # sde_utils.py:112-123
            ts = T + 2
            x = np.linspace(0, ts, ts + 1, dtype=f32)
            ac = np.cos(((x / f32(ts)) + f32(0.008)) / f32(1.008) * f32(math.pi * 0.5)) ** 2
            ac = (ac / ac[0]).astype(f32)
            thetas = (1 - ac[1:-1]).astype(f32)
        elif schedule == "linear":                 # sde_utils.py:101-110
            ts = T + 1
            scale = 1000 / ts
            thetas = np.linspace(scale * 0.0001, scale * 0.02, ts, dtype=f32)
        else:                                      # constant, sde_utils.py:93-99
            thetas = np.ones(T + 1, f32)
        self.thetas = thetas.astype(f32)
        self.sigmas = np.sqrt(f32(ms ** 2 * 2) * self.thetas).astype(f32)
        self.thetas_cumsum = (np.cumsum(self.thetas, dtype=f32) - self.thetas[0]).astype(f32)
        self.dt = f32(-1 / self.thetas_cumsum[-1] * f32(math.log(eps)))
        self.sigma_bars = np.sqrt(f32(ms ** 2) * (1 - np.exp(-2 * self.thetas_cumsum * self.dt))
                                  ).astype(f32)
        self.mu = None
        self.model = None

    def posterior_coeffs(self, t):
        """(x0 scale, term1, term2, std) for step t (sde_utils.py:205-225, 245-247)."""
        th, tc, tc1, dt = self.thetas[t], self.thetas_cumsum[t], self.thetas_cumsum[t - 1], self.dt
        ea = np.exp(tc * dt).astype(f32)
        A, B, C = np.exp(-th * dt), np.exp(-tc * dt), np.exp(-tc1 * dt)
        term1 = A * (1 - C ** 2) / (1 - B ** 2)
        term2 = C * (1 - A ** 2) / (1 - B ** 2)
        A2, B2, C2 = np.exp(-2 * th * dt), np.exp(-2 * tc * dt), np.exp(-2 * tc1 * dt)
        var = (1 - A2) * (1 - C2) / (1 - B2)
        std = np.exp(0.5 * np.log(np.maximum(var, f32(1e-20) * dt))) * f32(self.max_sigma)
        return f32(ea), f32(term1), f32(term2), f32(std)

    def noise_state(self, x, z):
        return (x + z * f32(self.max_sigma)).astype(f32)

    def posterior_step(self, x, eps, t, z):
        mu = self.mu
        ea, t1, t2, std = self.posterior_coeffs(t)
        x0 = (x - mu - self.sigma_bars[t] * eps) * ea + mu
        mean = t1 * (x - mu) + t2 * (x0 - mu) + mu
        return (mean + std * z).astype(f32)

    def sde_step(self, x, eps, t, z):
        """reverse_sde_step with score = -eps / sigma_bar (sde_utils.py:44-45,177-187)."""
        mu = self.mu
        score = -eps / self.sigma_bars[t]
        drift = (self.thetas[t] * (mu - x) - self.sigmas[t] ** 2 * score) * self.dt
        disp = self.sigmas[t] * (z * f32(math.sqrt(self.dt)))
        return (x - drift - disp).astype(f32)

    def reverse_posterior(self, xt, noises, T=None, **ctx):
        T = T or self.T
        x = xt.copy()
        for i, t in enumerate(range(T, 0, -1)):
            x = self.posterior_step(x, self.model(x, self.mu, t * self.sample_scale, **ctx), t, noises[i])
        return x

    def reverse_sde(self, xt, noises, T=None, **ctx):
        T = T or self.T
        x = xt.copy()
        for i, t in enumerate(range(T, 0, -1)):
            x = self.sde_step(x, self.model(x, self.mu, t * self.sample_scale, **ctx), t, noises[i])
        return x
