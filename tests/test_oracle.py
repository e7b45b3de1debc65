"""Pin the numpy oracle against fixtures produced by the reference itself (make_golden.py)."""
import numpy as np
import pytest

import oracle
from oracle import unet as OU, clip as OC, sde as OS, imgs as OI


def rel(a, b):
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


@pytest.mark.parametrize("tag", ["32x32", "30x34", "64x64"])
def test_unet_forward_matches_reference(golden, unet_sd, tag):
    g = golden(f"unet_fwd_nf64_{tag}.npz")
    out = OU.forward(unet_sd, g["xt"], g["mu"], float(g["t"]), g["text_context"], g["image_context"])
    assert out.shape == g["out"].shape
    assert rel(out, g["out"]) < 2e-5


def test_modules_match_reference(golden):
    from daclip_amd import synth
    g = golden("modules.npz")
    for tag in ("rb64", "rb96_32"):
        din = g[f"{tag}_x"].shape[1]
        dout = g[f"{tag}_y"].shape[1]
        spec = {"mlp.1.weight": (2 * dout, 256), "mlp.1.bias": (2 * dout,),
                "block1.proj.weight": (dout, din, 3, 3), "block2.proj.weight": (dout, dout, 3, 3)}
        if din != dout:
            spec["res_conv.weight"] = (dout, din, 1, 1)
        sd = synth.synth_state_dict(spec, seed=5)
        y = OU.resblock(sd, "", g[f"{tag}_x"], g[f"{tag}_t"])
        assert rel(y, g[f"{tag}_y"]) < 1e-5, tag
    spec = {"to_qkv.weight": (384, 64, 1, 1), "to_out.0.weight": (64, 128, 1, 1),
            "to_out.0.bias": (64,), "to_out.1.g": (1, 64, 1, 1)}
    sd = synth.synth_state_dict(spec, seed=5)
    assert rel(OU.linear_attention(sd, "", g["la_x"]), g["la_y"]) < 1e-5


def test_sde_tables_match_reference(golden):
    g = golden("sde_tables.npz")
    for name, sched in (("cos", "cosine"), ("lin", "linear")):
        s = OS.IRSDE(50, 100, sched, 0.005)
        for f in ("thetas", "sigmas", "thetas_cumsum", "sigma_bars"):
            np.testing.assert_allclose(getattr(s, f), g[f"{name}_{f}"], rtol=1e-5, atol=1e-6)  # cos: 1-ulp libm differences
        np.testing.assert_allclose(s.dt, g[f"{name}_dt"], rtol=2e-6)
    assert s.max_sigma == pytest.approx(float(g["max_sigma"]))


def test_posterior_loop_matches_reference(golden, unet_sd):
    """Full T=100 posterior loop at 16x16 with injected noise (parity of the whole sampler)."""
    g = golden("posterior_loop_16x16.npz")
    s = OS.IRSDE(50, 100, "cosine", 0.005)
    s.mu = g["lq"]
    s.model = lambda x, mu, t, **k: OU.forward(unet_sd, x, mu, t, **k)
    noisy = s.noise_state(g["lq"], g["noise_state"])
    np.testing.assert_allclose(noisy, g["noisy"], rtol=1e-6, atol=1e-7)
    ctx = dict(text_context=g["text_context"], image_context=g["image_context"])
    out = s.reverse_posterior(noisy, g["step_noise"], **ctx)
    assert rel(out, g["out"]) < 1e-3
    u8 = OI.tensor2img(out[0])
    assert np.mean(u8 != g["out_u8"]) < 0.01
    out3 = s.reverse_sde(noisy, g["step_noise"][:3], T=3, **ctx)
    assert rel(out3, g["out_sde3"]) < 1e-4


@pytest.mark.parametrize("name", ["daclip_small_encode.npz", "daclip_b32_encode.npz"])
def test_daclip_encode_matches_reference(golden, name):
    from daclip_amd import arch, synth
    g = golden(name)
    if "small" in name:
        v = arch.VisionConfig(image_size=64, patch_size=32, width=128, layers=3, embed_dim=64)
        t = arch.TextConfig(context_length=16, vocab_size=64, width=64, heads=2, layers=1)
    else:
        v, t = arch.VIT_B_32, arch.TEXT_B_32
    spec = {k: s for k, s in arch.daclip_state_spec(v, t).items()
            if "visual" in k}
    sd = synth.synth_state_dict(spec, seed=0)
    ic, dc = OC.encode_image(sd, g["img"])
    assert rel(ic, g["image_context"]) < 1e-4
    assert rel(dc, g["degra_context"]) < 1e-4


def test_img_metrics_match_reference(golden):
    g = golden("img_metrics.npz")
    assert np.array_equal(OI.tensor2img(g["a"]), g["ua"])
    assert np.array_equal(OI.tensor2img(g["b"]), g["ub"])
    assert OI.calculate_psnr(g["ua"], g["ub"]) == pytest.approx(float(g["psnr"]), abs=1e-12)


def test_sample_scale_loop_matches_reference(golden, unet_sd):
    """IRSDE(T=100, sample_T=50): 50-entry schedule, model at t * 2 (sde_utils.py:84-89, 302)."""
    g = golden("sampler_variants.npz")
    s = OS.IRSDE(50, 100, "cosine", 0.005, sample_T=50)
    np.testing.assert_allclose(s.thetas, g["st_thetas"], rtol=1e-5, atol=1e-6)
    assert s.sample_scale == 2.0
    s.mu = g["st_lq"]
    s.model = lambda x, mu, t, **k: OU.forward(unet_sd, x, mu, t, **k)
    out = s.reverse_posterior(g["st_x0"], g["st_steps"], text_context=g["st_tc"], image_context=g["st_ic"])
    assert rel(out, g["st_out"]) < 1e-3


def _selfctx_sd():
    from daclip_amd import arch, synth
    cfg = arch.UNetConfig(3, 3, 64, (1, 2, 4, 4), 256, True, True)
    return synth.synth_state_dict(arch.unet_state_spec(cfg), seed=1)


def test_selfctx_spec_matches_reference(golden):
    import json
    import os
    from daclip_amd import arch
    from conftest import GOLDEN
    ref = json.load(open(os.path.join(GOLDEN, "selfctx_state_spec.json")))
    ours = arch.unet_state_spec(arch.UNetConfig(3, 3, 64, (1, 2, 4, 4), 256, True, True))
    assert {k: list(v) for k, v in ours.items()} == ref


def test_image_context_none_matches_reference(golden):
    """image_context=None: attn2 is self-attention over norm2(x) (attention.py:174)."""
    g = golden("sampler_variants.npz")
    sd = _selfctx_sd()
    out = OU.forward(sd, g["sc_xt"], g["sc_mu"], 31.0, text_context=g["sc_tc"], image_context=None)
    assert rel(out, g["sc_fwd"]) < 2e-5
    out = OU.forward(sd, g["sc_xt"], g["sc_mu"], 7.0)
    assert rel(out, g["sc_fwd_notext"]) < 2e-5


def test_headline_encode_matches_reference(golden):
    """The real 256x256 image of the headline fixture: clip_transform (PIL restatement) is
    reproduced bit-exactly and the oracle encode matches the reference's contexts."""
    from daclip_amd import arch, synth
    from daclip_amd.preprocess import clip_transform
    g = golden("headline_256_t100.npz")
    img = clip_transform(g["rgb_u8"] / 255.0).unsqueeze(0).numpy()
    assert np.array_equal(img, g["img4clip"])
    spec = {k: s for k, s in arch.daclip_state_spec(arch.VIT_B_32, arch.TEXT_B_32).items() if "visual" in k}
    ic, dc = OC.encode_image(synth.synth_state_dict(spec, seed=0), g["img4clip"])
    assert rel(ic, g["image_context"]) < 1e-4
    assert rel(dc, g["degra_context"]) < 1e-4


@pytest.mark.parametrize("which", ["small", "b32"])
def test_plain_encode_matches_reference(golden, which):
    """encode_image(image) with the default control=False (daclip_model.py:54-55)."""
    from daclip_amd import arch, synth
    g = golden("daclip_plain_encode.npz")
    if which == "small":
        v = arch.VisionConfig(image_size=64, patch_size=32, width=128, layers=3, embed_dim=64)
        t = arch.TextConfig(context_length=16, vocab_size=64, width=64, heads=2, layers=1)
        img = synth.synth_noise((3, 3, 64, 64), seed=12, tag="img4clip_small")
    else:
        v, t = arch.VIT_B_32, arch.TEXT_B_32
        img = golden("daclip_b32_encode.npz")["img"]
    spec = {k: s for k, s in arch.daclip_state_spec(v, t).items() if k.startswith("clip.visual.")}
    out = OC.encode_image(synth.synth_state_dict(spec, seed=0), img, control=False)
    assert rel(out, g[which]) < 1e-4
