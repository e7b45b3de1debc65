"""LQGT paired-folder dataset, test phase (data/LQGT_dataset.py:75-148; data/util.py:68-85
read_img, util.get_image_paths). cv2 is absent offline: images are decoded with PIL and turned
into cv2.imread's layout (HWC, BGR, uint8 -> float32 [0,1]; grayscale -> HW1; alpha dropped).
Returns, like the reference: LQ / GT as RGB CHW float tensors, LQ_clip (clip_transform of the
LQ), and the paths."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch
from PIL import Image

from .preprocess import clip_transform

IMG_EXT = (".jpg", ".JPG", ".jpeg", ".JPEG", ".png", ".PNG", ".ppm", ".PPM", ".bmp", ".BMP", ".tif", ".tiff")


def get_image_paths(root: str) -> List[str]:
    """Sorted image files under root (recursive), data/util.py get_paths_from_images."""
    out = []
    for d, _, files in sorted(os.walk(root)):
        out += [os.path.join(d, f) for f in sorted(files) if f.endswith(IMG_EXT)]
    if not out:
        raise RuntimeError(f"{root} has no valid image file")
    return sorted(out)


def read_img(path: str) -> np.ndarray:
    """cv2.imread(IMREAD_UNCHANGED) / 255 as float32 HWC BGR (data/util.py:68-85)."""
    im = Image.open(path)
    a = np.asarray(im)
    if a.ndim == 2:
        a = a[:, :, None]
    else:
        a = a[:, :, :3][:, :, ::-1]                # RGB(A) -> BGR, alpha dropped
    return np.ascontiguousarray(a).astype(np.float32) / 255.0


class LQGTDataset:
    def __init__(self, dataroot_LQ: str, dataroot_GT: Optional[str] = None):
        self.LQ_paths = get_image_paths(dataroot_LQ)
        self.GT_paths = get_image_paths(dataroot_GT) if dataroot_GT else None
        if self.GT_paths is not None and len(self.GT_paths) != len(self.LQ_paths):
            raise RuntimeError(f"GT and LQ datasets have different number of images - "
                               f"{len(self.GT_paths)}, {len(self.LQ_paths)}.")

    def __len__(self):
        return len(self.LQ_paths)

    def __getitem__(self, i) -> Dict[str, object]:
        lq = read_img(self.LQ_paths[i])
        gt = read_img(self.GT_paths[i]) if self.GT_paths else None
        if lq.shape[2] == 3:
            lq = lq[:, :, [2, 1, 0]]
            gt = gt[:, :, [2, 1, 0]] if gt is not None else None
        out = {"LQ": torch.from_numpy(np.ascontiguousarray(lq.transpose(2, 0, 1))).float(),
               "LQ_clip": clip_transform(lq), "LQ_path": self.LQ_paths[i],
               "GT_path": self.GT_paths[i] if self.GT_paths else None}
        if gt is not None:
            out["GT"] = torch.from_numpy(np.ascontiguousarray(gt.transpose(2, 0, 1))).float()
        return out
