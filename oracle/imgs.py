"""Image output + metric restatement (CPU oracle; TEST INFRASTRUCTURE ONLY).

tensor2img / calculate_psnr follow universal-image-restoration/utils/img_utils.py:136-164,
182-190.
"""
from __future__ import annotations

import math

import numpy as np


def tensor2img(t):
    """[3,H,W] float RGB -> uint8 HWC BGR: clamp[0,1], x255, round-half-even, cast."""
    a = np.clip(np.asarray(t, np.float32).squeeze(), 0, 1)
    if a.ndim == 3:
        a = np.transpose(a[[2, 1, 0]], (1, 2, 0))
    return np.round(a * np.float32(255.0)).astype(np.uint8)


def calculate_psnr(img1, img2):
    mse = np.mean((img1.astype(np.float64) - img2.astype(np.float64)) ** 2)
    if mse == 0:
        return float("inf")
    return 20 * math.log10(255.0 / math.sqrt(mse))
