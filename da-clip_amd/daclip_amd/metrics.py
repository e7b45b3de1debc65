"""Image-quality metrics of the reference evaluation (host-side numpy, like the reference).

* calculate_psnr: utils/img_utils.py:182-189 (float64 MSE over all pixels, inf if equal).
* ssim / calculate_ssim: utils/img_utils.py:192-234. Gaussian window 11x11, sigma 1.5 (the
  normalised cv2.getGaussianKernel(11, 1.5) outer product), per-channel 'valid' filtering
  (cv2.filter2D followed by the [5:-5, 5:-5] crop, so the border mode never matters), C1/C2
  of the 8-bit range. For 3-channel images the reference evaluates ssim on the whole HxWx3
  array (three times) -- i.e. the mean over all channels' SSIM maps; restated as such.
  Parity with cv2 is UNPINNED (cv2 is absent offline); tests check an independent direct
  window sum and SSIM identities.
* bgr2ycbcr: data/util.py:189-210 (BT.601, MATLAB-compatible); pinned by
  tests/golden/img_metrics.npz. Unlike the reference it does not scale a float input in place.
"""
from __future__ import annotations

import math

import numpy as np

from .preprocess import calculate_psnr  # noqa: F401  (utils/img_utils.py:182-189)


def gaussian_window(size: int = 11, sigma: float = 1.5) -> np.ndarray:
    x = np.arange(size, dtype=np.float64) - (size - 1) / 2.0
    g = np.exp(-(x * x) / (2.0 * sigma * sigma))
    g /= g.sum()
    return np.outer(g, g)


def _filter_valid(img: np.ndarray, win: np.ndarray) -> np.ndarray:
    """Correlation of each channel with `win`, 'valid' region only (== filter2D + crop)."""
    k = win.shape[0]
    v = np.lib.stride_tricks.sliding_window_view(img, (k, k), axis=(0, 1))
    return np.einsum("ij...kl,kl->ij...", v, win) if img.ndim == 2 else np.einsum("ijckl,kl->ijc", v, win)


def ssim(img1: np.ndarray, img2: np.ndarray) -> float:
    c1, c2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    a, b = img1.astype(np.float64), img2.astype(np.float64)
    w = gaussian_window()
    mu1, mu2 = _filter_valid(a, w), _filter_valid(b, w)
    s1 = _filter_valid(a * a, w) - mu1 * mu1
    s2 = _filter_valid(b * b, w) - mu2 * mu2
    s12 = _filter_valid(a * b, w) - mu1 * mu2
    m = ((2 * mu1 * mu2 + c1) * (2 * s12 + c2)) / ((mu1 * mu1 + mu2 * mu2 + c1) * (s1 + s2 + c2))
    return float(m.mean())


def calculate_ssim(img1: np.ndarray, img2: np.ndarray) -> float:
    if img1.shape != img2.shape:
        raise ValueError("Input images must have the same dimensions.")
    if img1.ndim == 2:
        return ssim(img1, img2)
    if img1.ndim == 3:
        if img1.shape[2] == 3:
            return ssim(img1, img2)        # the reference's 3 identical calls, averaged
        if img1.shape[2] == 1:
            return ssim(np.squeeze(img1), np.squeeze(img2))
    raise ValueError("Wrong input image dimensions.")


def bgr2ycbcr(img: np.ndarray, only_y: bool = True) -> np.ndarray:
    in_type = img.dtype
    x = img.astype(np.float64) * (1.0 if in_type == np.uint8 else 255.0)
    if only_y:
        r = np.dot(x, [24.966, 128.553, 65.481]) / 255.0 + 16.0
    else:
        r = np.matmul(x, [[24.966, 112.0, -18.214], [128.553, -74.203, -93.786],
                          [65.481, -37.797, 112.0]]) / 255.0 + [16, 128, 128]
    r = r.round() if in_type == np.uint8 else r / 255.0
    return r.astype(in_type)


def crop(img: np.ndarray, border: int) -> np.ndarray:
    return img if border == 0 else img[border:-border, border:-border]


def image_metrics(out_u8: np.ndarray, gt_u8: np.ndarray, crop_border: int = 0) -> dict:
    """test.py:146-196 for one image: PSNR / SSIM on BGR uint8 (as [0,1] floats * 255) and
    PSNR_Y / SSIM_Y on the Y channel. LPIPS needs its pretrained net (absent): not computed."""
    sr, gt = out_u8 / 255.0, gt_u8 / 255.0
    res = {"psnr": calculate_psnr(crop(sr, crop_border) * 255, crop(gt, crop_border) * 255),
           "ssim": calculate_ssim(crop(sr, crop_border) * 255, crop(gt, crop_border) * 255)}
    if gt.ndim == 3 and gt.shape[2] == 3:
        sy, gy = bgr2ycbcr(sr, True), bgr2ycbcr(gt, True)
        res["psnr_y"] = calculate_psnr(crop(sy, crop_border) * 255, crop(gy, crop_border) * 255)
        res["ssim_y"] = calculate_ssim(crop(sy, crop_border) * 255, crop(gy, crop_border) * 255)
    return res
