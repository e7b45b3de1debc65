"""Host-side image preprocessing and output metrics (numpy / PIL, like the reference).

* clip_transform: predict.py:94-106 / data/util.py:87-93 — PIL uint8 -> Resize(224, BICUBIC)
  on the short side -> CenterCrop(224) -> ToTensor -> Normalize(OPENAI mean/std,
  open_clip/constants.py:1-2). torchvision is absent offline, so this restates its PIL path
  (F.resize with an int: short side = size, long side = int(size * long / short); center
  crop offsets round((H - s) / 2)); parity with torchvision itself is UNPINNED.
* tensor2img / calculate_psnr: utils/img_utils.py:136-164, 182-190.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from PIL import Image

OPENAI_DATASET_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_DATASET_STD = (0.26862954, 0.26130258, 0.27577711)


def _resize_short(img: Image.Image, size: int) -> Image.Image:
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    if short == size:
        return img
    new_short, new_long = size, int(size * long / short)
    nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
    return img.resize((nw, nh), Image.BICUBIC)


def _center_crop(img: Image.Image, size: int) -> Image.Image:
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def clip_transform(np_image: np.ndarray, resolution: int = 224) -> torch.Tensor:
    """HWC float RGB in [0,1] -> normalized [3, res, res] float32 tensor."""
    pil = Image.fromarray((np_image * 255).astype(np.uint8))
    return pil_transform(pil, resolution)


def pil_transform(pil: Image.Image, resolution: int = 224) -> torch.Tensor:
    img = _center_crop(_resize_short(pil.convert("RGB"), resolution), resolution)
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.array(OPENAI_DATASET_MEAN, np.float32)) / np.array(OPENAI_DATASET_STD, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


def image_transform(image_size: int = 224):
    """open_clip.transform.image_transform(is_train=False) equivalent for PIL inputs."""
    def f(pil):
        return pil_transform(pil, image_size)
    return f


def tensor2img(tensor, out_type=np.uint8, min_max=(0, 1)):
    t = tensor.squeeze().float().cpu().clamp(*min_max)
    t = (t - min_max[0]) / (min_max[1] - min_max[0])
    a = t.numpy()
    if a.ndim == 3:
        a = np.transpose(a[[2, 1, 0], :, :], (1, 2, 0))
    if out_type == np.uint8:
        a = (a * 255.0).round()
    return a.astype(out_type)


def calculate_psnr(img1, img2):
    img1 = img1.astype(np.float64)
    img2 = img2.astype(np.float64)
    mse = np.mean((img1 - img2) ** 2)
    if mse == 0:
        return float("inf")
    return 20 * math.log10(255.0 / math.sqrt(mse))


def make_grid(tensor: torch.Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    """torchvision.utils.make_grid (normalize=False) for [B,C,H,W] -> [C, H', W'] (host)."""
    t = tensor.detach().float().cpu()
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if t.size(1) == 1:
        t = torch.cat((t, t, t), 1)
    if t.size(0) == 1:
        return t.squeeze(0)
    n = t.size(0)
    xm = min(nrow, n)
    ym = (n + xm - 1) // xm
    h, w = t.size(2) + padding, t.size(3) + padding
    grid = torch.full((t.size(1), h * ym + padding, w * xm + padding), pad_value)
    k = 0
    for y in range(ym):
        for x in range(xm):
            if k >= n:
                break
            grid[:, y * h + padding:(y + 1) * h, x * w + padding:(x + 1) * w] = t[k]
            k += 1
    return grid


def save_image(tensor: torch.Tensor, fp: str, nrow: int = 8, padding: int = 2) -> None:
    """torchvision.utils.save_image(normalize=False): grid * 255 + 0.5, clamp, uint8 PNG."""
    grid = make_grid(tensor, nrow=nrow, padding=padding)
    arr = grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    Image.fromarray(arr).save(fp)

