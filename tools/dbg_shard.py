"""Batch-composition check of one UNet forward: B images at once vs each image alone, under
several kernel-choice overrides (dac_conv3_force / dac_conv2_force). Prints max |diff|."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch
from daclip_amd import synth, _lib
from daclip_amd.unet import ConditionalUNet
R = int(sys.argv[1]) if len(sys.argv) > 1 else 32
L = _lib.lib()
for dt in ("fp32",):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, device="cuda:0", dtype=dt)
    m.load_synthetic(0)
    B = 3
    xt = torch.from_numpy(synth.synth_images(B, R, R, seed=1)).cuda()
    mu = torch.from_numpy(synth.synth_images(B, R, R, seed=2)).cuda()
    c = torch.from_numpy(synth.synth_noise((B, 512), seed=3, tag="c")).cuda()
    for f3, f2 in ((-1, 0), (0, 0), (-1, 1), (0, 1), (-1, 4)):
        L.dac_conv3_force(f3); L.dac_conv2_force(f2)
        full = m(xt, mu, 37.0, text_context=c, image_context=c)
        d = 0.0
        for i in range(B):
            one = m(xt[i:i + 1], mu[i:i + 1], 37.0, text_context=c[i:i + 1], image_context=c[i:i + 1])
            d = max(d, (one - full[i:i + 1]).abs().max().item())
        print(f"{dt} R={R} conv3_force={f3} conv2_force={f2}: max|B=3 - B=1| = {d:.3e}", flush=True)
