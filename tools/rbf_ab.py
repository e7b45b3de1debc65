"""A/B of the fused ResBlock inside the UNet: the same forward with rbfuse forced on (2) and off
(0) must be bit-identical, per batch size. Prints the first differing level if any."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "da-clip_amd"))
from daclip_amd import _lib, arch, synth  # noqa: E402
from daclip_amd.unet import ConditionalUNet  # noqa: E402

lib = _lib.lib()
sd = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
dt = sys.argv[1] if len(sys.argv) > 1 else "fp16"
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
res = {}
for on in (0, 2):
    # A fresh handle per setting: plans (and the dry run's choices) are per handle and shape.
    lib.dac_rbfuse_enable(on)
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt)
    m.load_state_dict(sd)
    for B in (1, 2, 8):
        x = T(synth.synth_noise((B, 3, 256, 256), seed=95, tag="b8") * 0.3 + 0.5)
        mu = T(synth.synth_images(B, 256, 256, seed=96))
        tc = T(synth.synth_noise((B, 512), seed=97, tag="tc"))
        ic = T(synth.synth_noise((B, 512), seed=98, tag="ic"))
        res[on, B] = m(x, mu, 42.0, text_context=tc, image_context=ic).float().cpu()
    del m
for B in (1, 2, 8):
    a, b = res[0, B], res[2, B]
    d = (a - b).abs()
    print(f"B {B}: equal {torch.equal(a, b)} max|d| {d.max().item():.3e} n_diff {(d > 0).sum().item()} of {d.numel()}")
print("B1 vs B8[0] (pair):", torch.equal(res[0, 1][0], res[0, 8][0]), " (fused):", torch.equal(res[2, 1][0], res[2, 8][0]))
lib.dac_rbfuse_enable(1)
