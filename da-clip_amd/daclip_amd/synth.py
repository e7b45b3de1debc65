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
