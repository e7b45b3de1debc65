"""PSNR of the HIP restore vs the reference's restore on the golden T=100 posterior fixture
(tests/golden/posterior_loop_16x16.npz). GT stand-in: the LQ image (no GT ships with the
fixture); the metric that matters is the PSNR *difference* between HIP and reference outputs."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import numpy as np, torch
from daclip_amd import arch, synth
from daclip_amd.unet import ConditionalUNet
from daclip_amd.sde import IRSDE
from daclip_amd.preprocess import tensor2img, calculate_psnr
g = np.load(os.path.join(ROOT, "tests/golden/posterior_loop_16x16.npz"))
sd = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
gt = tensor2img(torch.from_numpy(g["lq"][0]))
ref_u8 = g["out_u8"]
for dt in ("fp32", "bf16"):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt)
    m.load_state_dict(sd)
    s = IRSDE(50, 100, schedule="cosine", eps=0.005); s.set_model(m); s.set_mu(T(g["lq"]))
    out = s.reverse_posterior(T(g["noisy"]), noises=T(g["step_noise"]), text_context=T(g["text_context"]),
                              image_context=T(g["image_context"]))
    u8 = tensor2img(out[0])
    p_ours, p_ref = calculate_psnr(u8, gt), calculate_psnr(ref_u8, gt)
    print(f"{dt}: PSNR(ours,gt)={p_ours:.6f} PSNR(ref,gt)={p_ref:.6f} delta={p_ours - p_ref:+.2e} "
          f"PSNR(ours,ref)={calculate_psnr(u8, ref_u8):.2f} u8 mismatch={np.mean(u8 != ref_u8):.4f}")
