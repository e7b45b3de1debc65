"""Precision probe (GPU): which part of the bf16 path moves the headline restore away from the
reference? Restores the headline fixture (B=1, 256^2, T=100) with encoder / UNet dtype
combinations and prints delta-PSNR vs the reference output, out max-rel error and PSNR of the
uint8 outputs against the reference's.
    python tools/prec_probe.py [combo ...]   combo = <enc dtype>/<unet dtype>, e.g. fp32/bf16
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from daclip_amd import arch, synth
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    combos = sys.argv[1:] or ["fp32/fp32", "bf16/fp32", "fp32/bf16", "bf16/bf16"]
    g = np.load(os.path.join(ROOT, "tests", "golden", "headline_256_t100.npz"))
    dev = torch.device("cuda", 0)
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0).to(dev)
    ns = torch.from_numpy(synth.synth_noise(tuple(lq.shape), seed=71, tag="hl_noise_state")).to(dev)
    zs = torch.from_numpy(synth.synth_noise((100,) + tuple(lq.shape), seed=72, tag="hl_steps")).to(dev)
    usd = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
    clips, unets = {}, {}
    for c in combos:
        e, u = c.split("/")
        if e not in clips:
            clips[e] = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, dtype=e, with_text=False)
            clips[e].load_synthetic(seed=0)
        if u not in unets:
            unets[u] = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=u)
            unets[u].load_state_dict(usd)
    ref = g["out"][0]
    for c in combos:
        e, u = c.split("/")
        ic, dc = clips[e].encode_image(torch.from_numpy(g["img4clip"]).to(dev), control=True)
        s = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
        s.set_model(unets[u])
        s.set_mu(lq)
        out = s.reverse_posterior(s.noise_state(lq, noise=ns), noises=zs, text_context=dc, image_context=ic)
        o = out[0].cpu().numpy()
        u8 = tensor2img(out[0])
        print(json.dumps({"combo": c,
                          "delta_db": calculate_psnr(u8, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"]),
                          "psnr_vs_ref_u8": calculate_psnr(u8, g["out_u8"]),
                          "out_rel": float(np.abs(o - ref).max() / np.abs(ref).max()),
                          "out_rms_rel": float(np.sqrt(np.mean((o - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))}),
              flush=True)


if __name__ == "__main__":
    main()
