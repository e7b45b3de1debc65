"""Batch evaluation over an LQ (+GT) folder pair: config/daclip-sde/test.py:87-234 on the
native path. Same-size images are restored together (one encode + one captured T-step loop
per batch; images are independent, so per-image results do not depend on the grouping).

    python -m daclip_amd.evaluate --opt test.yml --lq LQ_DIR [--gt GT_DIR] --out OUT_DIR
                                  [--synthetic] [--batch 8] [--dtype bf16]

Per image: restored PNG (test.py:131-138) and, with GT, PSNR / SSIM / PSNR_Y / SSIM_Y
(test.py:146-196). LPIPS needs its pretrained network, which is unavailable offline: not
computed (reported as None).
"""
from __future__ import annotations

import argparse
import json
import os
import time
from collections import OrderedDict, defaultdict
from typing import Optional

import numpy as np
import torch
from PIL import Image

from . import open_clip
from .data import LQGTDataset
from .metrics import image_metrics
from .models import create_model, parse_options
from .preprocess import tensor2img
from .sde import IRSDE


def _setup(opt: dict, device: str, dtype: str, synthetic: bool, clip_name: str):
    if synthetic:
        opt = dict(opt, path=dict(opt.get("path") or {}, pretrain_model_G=None))
    model = create_model(opt, device=device, dtype=dtype)
    if synthetic:
        clip = open_clip.create_model(clip_name, device=model.device, dtype=dtype)
        clip.load_synthetic(0)
    else:
        clip, _ = open_clip.create_model_from_pretrained(clip_name, pretrained=opt["path"]["daclip"],
                                                         device=model.device, dtype=dtype)
    s = opt["sde"]
    sde = IRSDE(max_sigma=s["max_sigma"], T=s["T"], schedule=s["schedule"], eps=s["eps"], device=model.device)
    sde.set_model(model.model)
    return model, clip, sde, s.get("sampling_mode", "posterior")


def resolve_crop_border(opt: dict, crop_border: Optional[int] = None) -> int:
    """The metric crop of config/daclip-sde/test.py:84, 150: `opt["crop_border"]` when set
    (non-zero), else `opt["degradation"]["scale"]` (4 in options/test.yml:20); an explicit
    argument overrides both. 0 means no crop (test.py:151-160)."""
    if crop_border is not None:
        return int(crop_border)
    cb = opt.get("crop_border")
    if cb:
        return int(cb)
    return int((opt.get("degradation") or {}).get("scale") or 0)


def evaluate(opt: dict, lq_dir: str, gt_dir: Optional[str], out_dir: str, batch: int = 8,
             device: str = "cuda", dtype: str = "fp32", synthetic: bool = False,
             clip_name: str = "daclip_ViT-B-32", crop_border: Optional[int] = None,
             suffix: str = "") -> dict:
    crop_border = resolve_crop_border(opt, crop_border)
    model, clip, sde, mode = _setup(opt, device, dtype, synthetic, clip_name)
    ds = LQGTDataset(lq_dir, gt_dir)
    os.makedirs(out_dir, exist_ok=True)
    groups = defaultdict(list)                       # same-size images restore together
    for i in range(len(ds)):
        groups[tuple(ds[i]["LQ"].shape)].append(i)
    per_image, times = OrderedDict(), []
    for _, idx in sorted(groups.items()):
        for k in range(0, len(idx), batch):
            items = [ds[i] for i in idx[k:k + batch]]
            lq = torch.stack([it["LQ"] for it in items])
            img4clip = torch.stack([it["LQ_clip"] for it in items]).to(model.device)
            with torch.no_grad():
                ic, dc = clip.encode_image(img4clip, control=True)
            noisy = sde.noise_state(lq)
            gt = torch.stack([it["GT"] for it in items]) if gt_dir else None
            model.feed_data(noisy, lq, gt, text_context=dc.float(), image_context=ic.float())
            torch.cuda.synchronize()
            t0 = time.time()
            model.test(sde, mode=mode, save_states=False)
            torch.cuda.synchronize()
            times.append((time.time() - t0) / len(items))
            vis = model.get_current_visuals(need_GT=gt_dir is not None)
            for j, it in enumerate(items):
                name = os.path.splitext(os.path.basename(it["GT_path"] or it["LQ_path"]))[0]
                out_u8 = tensor2img(vis["Outputs"][j])                    # BGR HWC uint8
                Image.fromarray(out_u8[:, :, ::-1]).save(os.path.join(out_dir, name + suffix + ".png"))
                rec = {"time_s": times[-1]}
                if gt_dir:
                    rec.update(image_metrics(out_u8, tensor2img(vis["GTs"][j]), crop_border))
                    rec["lpips"] = None
                per_image[name] = rec
    summary = {"images": len(per_image), "avg_time_s": float(np.mean(times)) if times else None}
    if gt_dir and per_image:
        for key in ("psnr", "ssim", "psnr_y", "ssim_y"):
            vals = [r[key] for r in per_image.values() if key in r]
            summary[key] = float(np.mean(vals)) if vals else None
    return {"per_image": per_image, "summary": summary}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--opt", required=True, help="options yml (config/daclip-sde/options/test.yml)")
    ap.add_argument("--lq", required=True)
    ap.add_argument("--gt", default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16", "bf16"])
    ap.add_argument("--synthetic", action="store_true", help="seeded synthetic weights (no checkpoints)")
    ap.add_argument("--clip", default="daclip_ViT-B-32")
    ap.add_argument("--crop-border", type=int, default=None,
                    help="pixels cropped before the metrics (default: test.py:150, opt crop_border else "
                         "degradation.scale)")
    a = ap.parse_args(argv)
    res = evaluate(parse_options(a.opt), a.lq, a.gt, a.out, a.batch, dtype=a.dtype, synthetic=a.synthetic,
                   clip_name=a.clip, crop_border=a.crop_border)
    print(json.dumps(res["summary"]))
    return res


if __name__ == "__main__":
    main()
