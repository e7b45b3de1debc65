"""Deterministic synthetic weights and inputs (no checkpoints exist offline).

Each tensor is drawn from its own numpy PCG64 stream seeded by (seed, crc32(key)), so the
value of one key never depends on which other keys exist, and the golden-fixture generator
(tests/golden/make_golden.py), the oracle and the HIP path all see bit-identical weights.
Scales follow PyTorch's default layer init (uniform ±1/sqrt(fan_in)) so activations stay
in the range a trained network produces; norm gains are 1 ± 0.1 so the affine paths are
exercised. Modules the reference zero-initialises (SpatialTransformer.proj_out,
ControlTransformer.zero_modules) get random values on purpose, so their paths are tested.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Mapping, Tuple

import numpy as np

from .arch import canonical_daclip_key


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def synth_tensor(key: str, shape: Tuple[int, ...], seed: int = 0) -> np.ndarray:
    r = _rng(seed, key)
    leaf = key.rsplit(".", 1)[-1]
    if len(shape) == 0:
        return np.array(np.log(1 / 0.07), dtype=np.float32)
    if leaf in ("class_embedding", "positional_embedding", "proj", "text_projection"):
        w = shape[-1] if leaf != "proj" else shape[0]
        return (r.standard_normal(shape) * w ** -0.5).astype(np.float32)
    if leaf == "prompt":
        return r.random(shape).astype(np.float32)          # torch.rand (DenoisingUNet_arch.py:59)
    if "token_embedding" in key:
        return (r.standard_normal(shape) * 0.02).astype(np.float32)
    if leaf == "g" or (leaf == "weight" and len(shape) == 1):
        return (1.0 + r.uniform(-0.1, 0.1, shape)).astype(np.float32)
    if leaf.endswith("bias"):
        return r.uniform(-0.05, 0.05, shape).astype(np.float32)
    fan_in = int(np.prod(shape[1:]))
    b = fan_in ** -0.5
    return r.uniform(-b, b, shape).astype(np.float32)


def synth_state_dict(spec: Mapping[str, Tuple[int, ...]], seed: int = 0,
                     canonical=canonical_daclip_key) -> Dict[str, np.ndarray]:
    """{key: float32 array}. Aliased keys (visual.* == clip.visual.*) get identical values."""
    return {k: synth_tensor(canonical(k), tuple(s), seed) for k, s in spec.items()}


def synth_images(n: int, h: int, w: int, seed: int = 0) -> np.ndarray:
    """[n,3,h,w] float32 in [0,1]: smooth gradients + texture, one stream per image."""
    out = np.empty((n, 3, h, w), np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    for i in range(n):
        r = _rng(seed + i, "image")
        base = np.stack([(0.3 + 0.4 * np.sin(3 * xx * (c + 1) + r.random() * 6)
                          * np.cos(2 * yy + c)) for c in range(3)])
        out[i] = np.clip(base + 0.08 * r.standard_normal((3, h, w)), 0, 1)
    return out


def synth_noise(shape: Iterable[int], seed: int = 0, tag: str = "noise") -> np.ndarray:
    return _rng(seed, tag).standard_normal(tuple(shape)).astype(np.float32)


# --------------------------------------------------------------------------- tracking weights
TRACK_T = 100
TRACK_KNOTS = np.arange(0, 256, 2)[:TRACK_T]      # time-embedding dims carrying the t hinges
TRACK_GAMMA = 10.0                                # hinge slope per unit t


def tracking_projection() -> np.ndarray:
    """A [3, 64, 3, 3]: the random 3x3 projection of the deep-path channels that forms D, each
    kernel zero-sum over its taps, so per-channel constants of the deep features (bias-driven)
    cancel and D is image-dependent texture with no colour cast."""
    A = synth_tensor("tracking.D", (3, 64, 3, 3), seed=0)
    return (A - A.mean(axis=(2, 3), keepdims=True)).astype(np.float32)


def tracking_state_dict(sd: Mapping[str, np.ndarray], w_g1: np.ndarray, w_g2: np.ndarray,
                        k: float) -> Dict[str, np.ndarray]:
    """Synthetic nf=64 UNet weights (ch_mult [1,2,4,8], context 512) under which the reference's
    T=100 posterior loop restores instead of diverging (the restoration fixture,
    tests/golden/make_golden.py gen_restore). With random weights eps does not track
    (x - mu)/sigma_bar_t, so the posterior's (x - mu) coefficient (~1.11 per step at t ~ 100,
    sde_utils.py:205-213, 245-247) multiplies up to 1/eps = 200 and the output saturates.
    These weights make the network predict

        eps = g1(t) (x - mu) - g2(t) D,    g1 = 1/sigma_bar_t,  g2 = exp(-theta_cumsum_t dt)/sigma_bar_t

    so that x0 = mu + D, where D = k * (3x3 projection A of the 64 deep-path channels entering
    final_res_block, tracking_projection()): every down / mid / up kernel shapes the output. Inside the architecture
    (DenoisingUNet_arch.py:118-174):
      * init_conv channels 0..2 copy xt - cond (7x7 centre tap 1);
      * time_mlp dims TRACK_KNOTS carry hinges GELU(GAMMA (i + 3/2 - t)), i = 0..T-1, from the
        lowest sinusoid frequency (sin(1e-4 t) ~ 1e-4 t, module_util.py:36-48); prompt_mlp and
        every ResBlock mlp read none of them, except the scale rows of final_res_block channels
        0..5 (weights w_g1, fitted to g1 - 1 at t = 1..T) and 6..11 (w_g2, to g2 - 1);
      * final_res_block.block1 channel pairs (2j, 2j+1) = +-(x - mu)_j, (6+2j, 7+2j) = +-D_j;
        block2 re-forms the pairs and final_conv takes differences: SiLU(z) - SiLU(-z) = z
        exactly, so neither nonlinearity distorts the path;
      * final_res_block.res_conv rows 0..11, final_conv columns 12..63 and its bias are zero.
    `w_g1`, `w_g2` (length T) and `k` are fitted by the fixture generator on the reference and
    stored in the fixture. Returns a new {key: float32 array}."""
    sd = {key: np.array(v, np.float32, copy=True) for key, v in sd.items()}
    T, kd = TRACK_T, TRACK_KNOTS
    other = np.setdiff1d(np.arange(256), kd)
    w1 = sd["time_mlp.1.weight"]
    w1[kd] = 0.0
    w1[kd, 31] = -TRACK_GAMMA * 1e4
    sd["time_mlp.1.bias"][kd] = TRACK_GAMMA * (np.arange(T) + 1.5)
    w3 = sd["time_mlp.3.weight"]
    w3[kd] = 0.0
    w3[kd, kd] = 1.0
    w3[np.ix_(other, kd)] = 0.0
    sd["time_mlp.3.bias"][kd] = 0.0
    sd["prompt_mlp.weight"][kd] = 0.0
    sd["prompt_mlp.bias"][kd] = 0.0
    for key in sd:
        if key.endswith(".mlp.1.weight"):
            sd[key][:, kd] = 0.0
    ic = sd["init_conv.weight"]
    ic[:3] = 0.0
    p = "final_res_block."
    c1, c2 = sd[p + "block1.proj.weight"], sd[p + "block2.proj.weight"]
    c1[:12], c2[:12] = 0.0, 0.0
    sd[p + "res_conv.weight"][:12] = 0.0
    fc = sd["final_conv.weight"]
    fc[:] = 0.0
    sd["final_conv.bias"][:] = 0.0
    A = tracking_projection()
    for j in range(3):
        ic[j, j, 3, 3] = 1.0
        c1[2 * j, 64 + j, 1, 1], c1[2 * j + 1, 64 + j, 1, 1] = 1.0, -1.0
        c1[6 + 2 * j, :64], c1[7 + 2 * j, :64] = k * A[j], -k * A[j]
        for q in (2 * j, 6 + 2 * j):
            c2[q, q, 1, 1], c2[q, q + 1, 1, 1] = 1.0, -1.0
            c2[q + 1, q, 1, 1], c2[q + 1, q + 1, 1, 1] = -1.0, 1.0
        fc[j, 2 * j, 1, 1], fc[j, 2 * j + 1, 1, 1] = 1.0, -1.0
        fc[j, 6 + 2 * j, 1, 1], fc[j, 7 + 2 * j, 1, 1] = -1.0, 1.0
    mw, mb = sd[p + "mlp.1.weight"], sd[p + "mlp.1.bias"]
    mw[:12], mb[:12] = 0.0, 0.0
    mw[64:76], mb[64:76] = 0.0, 0.0                  # their shifts
    for r in range(6):
        mw[r, kd] = w_g1
        mw[6 + r, kd] = w_g2
    return sd
