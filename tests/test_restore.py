"""North-star PSNR bar on a restoration the reference actually performs.

tests/golden/restore_rain_256_t100.npz is the reference's predict.py:58-91 flow run in the
fixture builder (make_golden.py gen_restore) on the 256x256 centre crop of images/3_rain.png
(BASELINE configs[0]): seed-0 ViT-B/32 DaCLIP, ConditionalUNet nf=64 with the tracking weights
of synth.tracking_state_dict (eps follows (x - mu)/sigma_bar_t, so the reference's own T=100
posterior loop converges to LQ + D instead of diverging; 98.5 % of its output pixels lie in
(0, 1), 27.1 dB against the LQ), injected noise, fp32 CPU. The HIP path restores it through
the C ABI (graph-captured loop) and is held, per dtype, to:
  * |PSNR(ours, LQ) - PSNR(reference, LQ)| < 1e-3 dB on uint8 (tensor2img, calculate_psnr);
  * the fraction of uint8 values that differ from the reference's, and the largest float
    error on the pixels the reference leaves in (0, 1) (absolute, not normalised).
fp8 (BASELINE configs[4]) is measured on the same fixture and bounded separately.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def record(name, **kv):
    print(name, json.dumps(kv))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "restore_metrics.jsonl"), "a") as f:
            f.write(json.dumps({"test": name, **kv}) + "\n")


def lq_of(g):
    return torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0)   # predict.py:73-75


def unet(dtype, sd):
    from daclip_amd.unet import ConditionalUNet
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dtype)
    m.load_state_dict(sd)
    return m


def contexts(dtype, g, B):
    from daclip_amd import arch
    from daclip_amd.open_clip import DaCLIP
    clip = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, dtype=dtype, with_text=False)
    clip.load_synthetic(seed=0)
    img = torch.from_numpy(g["img4clip"]).cuda().expand(B, -1, -1, -1).contiguous()
    return clip.encode_image(img, control=True)


def restore(dtype, g, sd, noise, B):
    """predict.py:63-86 on the HIP path for B copies of the fixture image."""
    from daclip_amd.sde import IRSDE
    ic, dc = contexts(dtype, g, B)
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    sde.set_model(unet(dtype, sd))
    lqb = lq_of(g).cuda().expand(B, -1, -1, -1).contiguous()
    noisy = sde.noise_state(lqb, noise=torch.from_numpy(noise["n0"]).cuda().expand(B, -1, -1, -1))
    sde.set_mu(lqb)
    z = torch.from_numpy(noise["steps"]).cuda().expand(-1, B, -1, -1, -1).contiguous()
    out = sde.reverse_posterior(noisy, noises=z, text_context=dc, image_context=ic)
    torch.cuda.synchronize()
    return ic.cpu().numpy(), dc.cpu().numpy(), out.cpu().numpy()


def metrics(g, out0):
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    ref = g["out"][0]
    u8 = tensor2img(torch.from_numpy(out0))
    inr = (ref > 0) & (ref < 1)
    return dict(delta_psnr_db=float(calculate_psnr(u8, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"])),
                psnr_vs_ref_u8=float(calculate_psnr(u8, g["out_u8"])),
                u8_mismatch=float(np.mean(u8 != g["out_u8"])),
                u8_max_diff=int(np.abs(u8.astype(int) - g["out_u8"].astype(int)).max()),
                inrange_max_abs=float(np.abs(out0 - ref)[inr].max()),
                inrange_rms=float(np.sqrt(np.mean((out0 - ref)[inr] ** 2))))


# (B, ctx rel bound, dPSNR bound dB, u8 mismatch bound, in-range max-abs bound)
BARS = {"fp32": (2, 1e-4, 1e-3, 2e-3, 5e-4),
        "fp16": (8, 5e-3, 1e-3, 0.06, 5e-3),
        "bf16": (8, 2e-2, 1e-2, 0.35, 2e-2)}


@pytest.mark.parametrize("dtype", ["fp32", "fp16", "bf16"])
def test_restore_matches_reference(restore_fixture, dtype):
    g, sd, noise = restore_fixture
    B, ctx_tol, dpsnr, mism, maxabs = BARS[dtype]
    ic, dc, out = restore(dtype, g, sd, noise, B)
    for b in range(1, B):                               # every copy restores identically
        assert np.array_equal(out[b], out[0]), b
    ctx = max(float(np.abs(ic[0] - g["image_context"][0]).max() / np.abs(g["image_context"][0]).max()),
              float(np.abs(dc[0] - g["degra_context"][0]).max() / np.abs(g["degra_context"][0]).max()))
    m = metrics(g, out[0])
    record(f"restore_{dtype}", ctx_rel=ctx, **m)
    assert ctx < ctx_tol
    assert abs(m["delta_psnr_db"]) < dpsnr              # north-star bar
    assert m["u8_mismatch"] < mism
    assert m["inrange_max_abs"] < maxabs


def test_restore_fp8_measured(restore_fixture):
    """fp8 handles (BASELINE configs[4]): the 16-bit (bf16) kernels with the 64 -> 64 ResBlock
    block2 convs on e4m3 MX operands (block1 writes h as e4m3 + per-(pixel, 32-channel)
    exponents, conv3q.hip) and the ViT GEMMs on e4m3 MX weights (conv8.hip). dPSNR measured and
    bounded at 2x the measurement: +0.059 dB, 51.9 dB against the reference's uint8, in-range
    max-abs 0.053 (round 3's all-conv8 UNet: -2.31 dB, max-abs 0.156)."""
    g, sd, noise = restore_fixture
    _, _, out = restore("fp8", g, sd, noise, 2)
    assert np.array_equal(out[1], out[0])
    assert np.isfinite(out).all()
    m = metrics(g, out[0])
    record("restore_fp8", **m)
    assert abs(m["delta_psnr_db"]) < 0.12
    assert m["inrange_max_abs"] < 0.11


def test_last_step_from_reference_state(restore_fixture):
    """One UNet forward + posterior update from the state the reference's loop reached at t=1
    (x_t1): isolates the network from trajectory drift."""
    from daclip_amd.sde import IRSDE
    g, sd, noise = restore_fixture
    m = unet("fp32", sd)
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    lq = lq_of(g).cuda()
    x = torch.from_numpy(g["x_t1"]).cuda()
    eps = m(x, lq, 1.0, text_context=torch.from_numpy(g["degra_context"]).cuda(),
            image_context=torch.from_numpy(g["image_context"]).cuda())
    out = sde.step(0, x, eps, lq, torch.from_numpy(noise["steps"][99]).cuda(), 1).cpu().numpy()
    err = float(np.abs(out - g["out"]).max())
    record("restore_last_step_fp32", max_abs=err)
    assert err < 1e-4                                 # fp32 summation order (0.03 levels)


@pytest.mark.parametrize("dtype", ["fp32", "fp16", "bf16"])
def test_reverse_sde_full_length(restore_fixture, dtype):
    """reverse_sde (mode='sde', sde_utils.py:261-277) for all T=100 steps at 64x64 against the
    reference run in the same fixture (only 3 steps were compared before)."""
    from daclip_amd.sde import IRSDE
    g, sd, noise = restore_fixture
    lq = lq_of(g)[:, :, 96:160, 96:160].contiguous().cuda()
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    sde.set_model(unet(dtype, sd))
    sde.set_mu(lq)
    noisy = sde.noise_state(lq, noise=torch.from_numpy(noise["n0_64"]).cuda())
    out = sde.reverse_sde(noisy, noises=torch.from_numpy(noise["steps_64"]).cuda(),
                          text_context=torch.from_numpy(g["degra_context"]).cuda(),
                          image_context=torch.from_numpy(g["image_context"]).cuda()).cpu().numpy()
    err = float(np.abs(out - g["out_sde64"]).max())
    record(f"reverse_sde64_{dtype}", max_abs=err)
    assert err < {"fp32": 2e-4, "fp16": 5e-3, "bf16": 2e-2}[dtype]


OPT = {
    "model": "denoising",
    "sde": {"max_sigma": 50, "T": 100, "schedule": "cosine", "eps": 0.005, "sampling_mode": "posterior"},
    "network_G": {"which_model_G": "ConditionalUNet",
                  "setting": {"in_nc": 3, "out_nc": 3, "nf": 64, "ch_mult": [1, 2, 4, 8],
                              "context_dim": 512, "use_degra_context": True, "use_image_context": True}},
}


@pytest.mark.parametrize("dtype", ["fp32", "fp16", "bf16"])
def test_predictor_chain_matches_reference(restore_fixture, tmp_path, dtype):
    """Predictor.setup/predict (predict.py:34-91) -> create_model / load_network
    (base_model.py:92-105, a module.-prefixed checkpoint file) -> DenoisingModel.feed_data /
    test / get_current_visuals (denoising_model.py:121-173) -> tensor2img, with the reference's
    injected noises, against the reference's uint8 output."""
    from daclip_amd.predict import Predictor
    from daclip_amd.preprocess import calculate_psnr
    g, sd, noise = restore_fixture
    ck = tmp_path / "universal-ir.pth"
    torch.save({"module." + k: torch.from_numpy(v) for k, v in sd.items()}, ck)
    opt = dict(OPT, path={"pretrain_model_G": str(ck), "strict_load": True})
    p = Predictor()
    p.setup(opt, dtype=dtype, synthetic_clip=True)
    bgr = np.ascontiguousarray(g["rgb_u8"][:, :, ::-1])            # cv2.imread order
    out = p.predict(bgr, noise=torch.from_numpy(noise["n0"]), noises=torch.from_numpy(noise["steps"]))
    assert out.shape == (256, 256, 3) and out.dtype == np.uint8
    d = float(calculate_psnr(out, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"]))
    mism = float(np.mean(out != g["out_u8"]))
    record(f"predictor_{dtype}", delta_psnr_db=d, u8_mismatch=mism)
    assert abs(d) < BARS[dtype][2]
    assert mism < BARS[dtype][3]
