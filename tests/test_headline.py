"""The benchmarked configuration (256x256, T=100 posterior, ViT-B/32 DA-CLIP + nf=64 UNet)
pinned end to end against the reference itself, run on a real image in the fixture builder
(tests/golden/make_golden.py gen_headline: predict.py:58-91 on images/00006.jpg with seeded
weights and injected noise). The HIP path restores B=8 copies through the captured graph loop.

North-star bar: restored output within 1e-3 dB PSNR of the reference CPU path. The fixture
has no ground truth, so PSNR is taken against the LQ input (as the reference's predict flow
would be scored on an LQ-only image). With seeded random weights the reference's loop
diverges (|out| up to 273, 99.3 % of the pixels clamp in tensor2img), so this fixture says
little about the PSNR bar: that is held on the restoration fixture instead (test_restore.py).
Here the float output is compared, and the error on the 0.7 % of pixels in (0, 1) is bounded.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 8
# Seeds of the injected noises, as in make_golden.py headline_noise().
NOISE_STATE = dict(seed=71, tag="hl_noise_state")
STEPS = dict(seed=72, tag="hl_steps")
T_STEPS = 100


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def record(name, **kv):
    """Measured values go to stdout and, on a GPU box, to gpurun_out/headline_metrics.jsonl."""
    print(name, json.dumps(kv))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "headline_metrics.jsonl"), "a") as f:
            f.write(json.dumps({"test": name, **kv}) + "\n")


@pytest.fixture(scope="module")
def headline(golden):
    from daclip_amd import synth
    g = golden("headline_256_t100.npz")
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0)   # predict.py:73-75
    n0 = torch.from_numpy(synth.synth_noise(tuple(lq.shape), **NOISE_STATE))
    steps = torch.from_numpy(synth.synth_noise((T_STEPS,) + tuple(lq.shape), **STEPS))
    return g, lq, n0, steps


def restore(dtype, g, lq, n0, steps, unet_sd):
    """predict.py:63-86 on the HIP path for B copies of the fixture image."""
    from daclip_amd import arch
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    clip = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, dtype=dtype, with_text=False)
    clip.load_synthetic(seed=0)
    img = torch.from_numpy(g["img4clip"]).cuda().expand(B, -1, -1, -1).contiguous()
    ic, dc = clip.encode_image(img, control=True)
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dtype)
    unet.load_state_dict(unet_sd)
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    sde.set_model(unet)
    lqb = lq.cuda().expand(B, -1, -1, -1).contiguous()
    noisy = sde.noise_state(lqb, noise=n0.cuda().expand(B, -1, -1, -1))
    sde.set_mu(lqb)
    z = steps.cuda().expand(-1, B, -1, -1, -1).contiguous()
    out = sde.reverse_posterior(noisy, noises=z, text_context=dc, image_context=ic)
    torch.cuda.synchronize()
    return ic.cpu().numpy(), dc.cpu().numpy(), out.cpu().numpy()


def check(name, g, ic, dc, out, ctx_tol, out_tol, unsat_tol):
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    assert rel(ic[0], g["image_context"][0]) < ctx_tol
    assert rel(dc[0], g["degra_context"][0]) < ctx_tol
    for b in range(1, B):                               # every copy restores identically
        assert np.array_equal(out[b], out[0]), b
    ref = g["out"][0]
    r = rel(out[0], ref)
    u8 = tensor2img(torch.from_numpy(out[0]))
    lq_u8 = g["lq_u8"]
    d_psnr = calculate_psnr(u8, lq_u8) - calculate_psnr(g["out_u8"], lq_u8)
    unsat = (ref > 0) & (ref < 1)
    record(name, ctx_rel=max(rel(ic[0], g["image_context"][0]), rel(dc[0], g["degra_context"][0])),
           out_rel=r, delta_psnr_db=d_psnr, psnr_vs_ref_u8=calculate_psnr(u8, g["out_u8"]),
           u8_mismatch=float(np.mean(u8 != g["out_u8"])), unsaturated_frac=float(unsat.mean()),
           unsat_max_abs=float(np.abs(out[0] - ref)[unsat].max()))
    assert abs(d_psnr) < 1e-3                           # north-star bar
    assert r < out_tol
    # the bound on the pixels this saturated fixture leaves in (0, 1), absolute
    assert float(np.abs(out[0] - ref)[unsat].max()) < unsat_tol


def test_headline_fp32_matches_reference(headline, unet_sd):
    g, lq, n0, steps = headline
    ic, dc, out = restore("fp32", g, lq, n0, steps, unet_sd)
    check("headline_fp32", g, ic, dc, out, ctx_tol=1e-4, out_tol=1e-3, unsat_tol=1e-2)


def test_headline_fp16_matches_reference(headline, unet_sd):
    """fp16, the bench's headline dtype (bench.py --dtype fp16, the default): the 1e-3 dB bar,
    every copy identical, and float bounds at least as tight as bf16's (fp16's significand is 8x
    finer; the encoder contexts carry fp16 activation rounding)."""
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    g, lq, n0, steps = headline
    ic, dc, out = restore("fp16", g, lq, n0, steps, unet_sd)
    check("headline_fp16", g, ic, dc, out, ctx_tol=5e-3, out_tol=8e-4, unsat_tol=0.1)
    assert calculate_psnr(tensor2img(torch.from_numpy(out[0])), g["out_u8"]) > 50.0


def test_headline_bf16_matches_reference(headline, unet_sd):
    """BASELINE configs[1]'s dtype (measured under the bench's `modes`). Measured: dPSNR 2.9e-4 dB, 55.9 dB against the reference's uint8
    output, float max-rel 3.2e-4 (bf16 weights with sum-keeping rounding; split-precision
    init_conv / final_conv / final_res_block.res_conv, engine.cpp)."""
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    g, lq, n0, steps = headline
    ic, dc, out = restore("bf16", g, lq, n0, steps, unet_sd)
    check("headline_bf16", g, ic, dc, out, ctx_tol=2e-2, out_tol=8e-4, unsat_tol=0.25)
    assert calculate_psnr(tensor2img(torch.from_numpy(out[0])), g["out_u8"]) > 50.0


def test_headline_fp8_psnr(headline, unet_sd):
    """fp8 handles (BASELINE configs[4]: e4m3 ResBlock block2 convs + ViT GEMMs) on the same
    fixture: the PSNR delta is measured and bounded at 2x (measured: dPSNR 1.2e-3 dB, 41.6 dB
    against the reference's uint8 output, float max-rel 1.5e-3); the run must stay finite and
    batch-invariant."""
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    g, lq, n0, steps = headline
    ic, dc, out = restore("fp8", g, lq, n0, steps, unet_sd)
    for b in range(1, B):
        assert np.array_equal(out[b], out[0]), b
    assert np.isfinite(out).all()
    u8 = tensor2img(torch.from_numpy(out[0]))
    d_psnr = calculate_psnr(u8, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"])
    record("headline_fp8", delta_psnr_db=d_psnr, psnr_vs_ref_u8=calculate_psnr(u8, g["out_u8"]),
           out_rel=rel(out[0], g["out"][0]), ctx_rel=max(rel(ic[0], g["image_context"][0]),
                                                          rel(dc[0], g["degra_context"][0])))
    assert abs(d_psnr) < 2.5e-3
    assert rel(out[0], g["out"][0]) < 3e-3
