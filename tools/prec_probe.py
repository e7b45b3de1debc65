"""Precision probe (GPU): which part of the bf16 path moves the restoration fixture
(tests/golden/restore_rain_256_t100.npz) away from the reference? One configuration per
process (the DAC_EMU_W / DAC_EMU_A role masks of engine.cpp are read once):
    [DAC_EMU_W=mask] [DAC_EMU_A=mask] python tools/prec_probe.py <enc dtype> <unet dtype> [label]
Prints one JSON line: dPSNR vs the reference on the LQ, uint8 mismatch, float error RMS on the
in-range pixels, and the error's regression on the restoration D = ref - LQ (scale error)."""
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
    e, u = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else f"{e}/{u}"
    g = np.load(os.path.join(ROOT, "tests", "golden", "restore_rain_256_t100.npz"))
    dev = torch.device("cuda", 0)
    sd = synth.tracking_state_dict(synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), 0),
                                   g["w_g1"], g["w_g2"], float(g["k"]))
    mi = os.environ.get("PROBE_MIXED")
    if mi is not None:
        # image `mi` of the mixed real-image fixture (tests/golden/mixed8_256_t100.npz), with its
        # slice of the batch's injected noise (tests/test_mixed.py mixed_noise)
        i = int(mi)
        m = np.load(os.path.join(ROOT, "tests", "golden", "mixed8_256_t100.npz"))
        n0 = synth.synth_noise((8, 3, 256, 256), seed=91, tag="mx_noise_state")[i:i + 1]
        st = synth.synth_noise((100, 8, 3, 256, 256), seed=92, tag="mx_steps")[:, i:i + 1]
        g = {"rgb_u8": m["rgb_u8"][i], "img4clip": m["img4clip"][i:i + 1], "out": m["out"][i:i + 1],
             "out_u8": m["out_u8"][i], "lq_u8": m["lq_u8"][i]}
        ns, zs = torch.from_numpy(n0).to(dev), torch.from_numpy(np.ascontiguousarray(st)).to(dev)
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0).to(dev)
    if mi is None:
        ns = torch.from_numpy(synth.synth_noise(tuple(lq.shape), seed=91, tag="rs_noise_state")).to(dev)
        zs = torch.from_numpy(synth.synth_noise((100,) + tuple(lq.shape), seed=92, tag="rs_steps")).to(dev)
    clip = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, dtype=e, with_text=False)
    clip.load_synthetic(seed=0)
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=u)
    unet.load_state_dict(sd)
    ic, dc = clip.encode_image(torch.from_numpy(g["img4clip"]).to(dev), control=True)
    s = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    s.set_model(unet)
    s.set_mu(lq)
    out = s.reverse_posterior(s.noise_state(lq, noise=ns), noises=zs, text_context=dc, image_context=ic)
    o = out[0].cpu().numpy().astype(np.float64)
    ref = g["out"][0].astype(np.float64)
    u8 = tensor2img(out[0])
    err = o - ref
    D = ref - lq[0].cpu().numpy()
    inr = (ref > 0) & (ref < 1)
    if os.environ.get("PROBE_SAVE"):
        np.save(os.path.join(ROOT, "gpurun_out", f"probe_{label.replace('/', '_')}.npy"), o.astype(np.float32))
    print(json.dumps({"label": label, "emu_w": os.environ.get("DAC_EMU_W"), "emu_a": os.environ.get("DAC_EMU_A"),
                      "delta_db": float(calculate_psnr(u8, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"])),
                      "u8_mismatch": float(np.mean(u8 != g["out_u8"])),
                      "err_rms": float(np.sqrt(np.mean(err[inr] ** 2))),
                      "scale_err": float((err * D).sum() / (D * D).sum()),
                      "corr": float(np.corrcoef(err.ravel(), D.ravel())[0, 1])}), flush=True)


if __name__ == "__main__":
    main()
