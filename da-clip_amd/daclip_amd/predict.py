"""predict.py mirror (Predictor.setup / predict, predict.py:34-91), plus a batched variant.

setup(): create_model(opt) -> native ConditionalUNet; open_clip.create_model_from_pretrained
("daclip_ViT-B-32", pretrained=opt["path"]["daclip"]) -> native DaCLIP; IRSDE(**opt["sde"])
with sde.set_model(model.model). predict(): BGR uint8 -> RGB [0,1] -> clip_transform ->
encode_image(control=True) -> noise_state -> feed_data -> test(sde) -> tensor2img (BGR uint8).

`predict_batch` restores B images in one pass (one encode + one captured loop for the whole
batch) and returns all of them; images must share one size. With no checkpoint on the box,
`synthetic=True` loads the seeded synthetic weights of both networks (`synthetic_clip` alone
keeps a UNet checkpoint from opt while the encoder is synthetic). Both predict entry points
take optional injected noises (the noise_state draw and the per-step draws) so the chain can
be pinned against the reference run with the same noises.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np
import torch
from PIL import Image

from . import open_clip
from .models import create_model, parse_options
from .preprocess import clip_transform, tensor2img
from .sde import IRSDE


def imread_bgr(path: str) -> np.ndarray:
    """cv2.imread(path) equivalent for 8-bit RGB files (PIL decode, channel order BGR)."""
    a = np.asarray(Image.open(path).convert("RGB"))
    return np.ascontiguousarray(a[:, :, ::-1])


class Predictor:
    def setup(self, opt: Union[str, dict], daclip_path: Optional[str] = None, device="cuda",
              dtype: str = "fp32", synthetic: bool = False,
              synthetic_clip: Optional[bool] = None) -> None:
        opt = parse_options(opt) if isinstance(opt, str) else dict(opt)
        if synthetic:
            opt["path"] = dict(opt.get("path") or {}, pretrain_model_G=None)
        self.model = create_model(opt, device=device, dtype=dtype)
        self.device = self.model.device
        if synthetic if synthetic_clip is None else synthetic_clip:
            self.clip_model = open_clip.create_model("daclip_ViT-B-32", device=self.device, dtype=dtype)
            self.clip_model.load_synthetic(0)
        else:
            path = daclip_path or opt["path"]["daclip"]
            self.clip_model, _ = open_clip.create_model_from_pretrained(
                "daclip_ViT-B-32", pretrained=path, device=self.device, dtype=dtype)
        s = opt["sde"]
        self.sde = IRSDE(max_sigma=s["max_sigma"], T=s["T"], schedule=s["schedule"], eps=s["eps"],
                         device=self.device)
        self.sde.set_model(self.model.model)
        self.mode = s.get("sampling_mode", "posterior")

    def _contexts(self, images_rgb01: Sequence[np.ndarray]):
        img4clip = torch.stack([clip_transform(im) for im in images_rgb01]).to(self.device)
        with torch.no_grad():
            ic, dc = self.clip_model.encode_image(img4clip, control=True)
        return ic.float(), dc.float()

    def predict_batch(self, images_bgr: Sequence[np.ndarray], noise: Optional[torch.Tensor] = None,
                      noises: Optional[torch.Tensor] = None) -> List[np.ndarray]:
        """predict.py:62-91 for B same-size images. `noise` [B,3,H,W] / `noises` [T,B,3,H,W]
        optionally replace the noise_state and per-step randn_like draws."""
        rgb = [im[:, :, [2, 1, 0]] / 255.0 for im in images_bgr]
        ic, dc = self._contexts(rgb)
        lq = torch.stack([torch.tensor(im, dtype=torch.float32).permute(2, 0, 1) for im in rgb])
        noisy = self.sde.noise_state(lq, noise=noise)
        self.model.feed_data(noisy, lq, text_context=dc, image_context=ic)
        self.model.test(self.sde, mode=self.mode, noises=noises)
        out = self.model.get_current_visuals(need_GT=False)["Outputs"]
        if not torch.isfinite(out).all():
            # 16-bit storage (fp16 saturates at 65504) must never turn into silent garbage pixels.
            raise RuntimeError(f"Predictor: non-finite restored output ({self.model.model.dtype} handles)")
        return [tensor2img(o) for o in out]

    def predict(self, image: Union[str, np.ndarray], noise: Optional[torch.Tensor] = None,
                noises: Optional[torch.Tensor] = None) -> np.ndarray:
        """One image (path or BGR uint8 HWC) -> restored BGR uint8 HWC."""
        im = imread_bgr(image) if isinstance(image, str) else image
        return self.predict_batch([im], noise=noise, noises=noises)[0]
