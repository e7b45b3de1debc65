"""Batch-invariance probe: UNet forward of B images vs each image alone, per dtype / batch /
switch; prints the max |difference| (0 = bit-identical). python tools/inv_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch  # noqa: E402
from daclip_amd import arch, synth  # noqa: E402
from daclip_amd.unet import ConditionalUNet  # noqa: E402

sd = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
for dt, B, env in [("fp16", 16, {}), ("bf16", 16, {}), ("bf16", 8, {}), ("fp8", 8, {}), ("fp8", 16, {}),
                   ("fp8", 16, {"DAC_Q8": "0"}), ("fp8", 2, {})]:
    for k in ("DAC_Q8",):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt)
    m.load_state_dict(sd)
    x = T(synth.synth_noise((B, 3, 256, 256), seed=101, tag="b16") * 0.3 + 0.5)
    mu = T(synth.synth_images(B, 256, 256, seed=102))
    tc = T(synth.synth_noise((B, 512), seed=103, tag="tc"))
    ic = T(synth.synth_noise((B, 512), seed=104, tag="ic"))
    full = m(x, mu, 42.0, text_context=tc, image_context=ic)
    d = []
    for i in (0, B - 1):
        one = m(x[i:i + 1], mu[i:i + 1], 42.0, text_context=tc[i:i + 1], image_context=ic[i:i + 1])
        d.append((one - full[i:i + 1]).abs().max().item())
    print(dt, B, env, "max|diff| per image", d, flush=True)
    del m
    torch.cuda.empty_cache()
