"""Wild-IR (§8f rank 3, BASELINE config 4 model): ConditionalUNet(scale=0.5, context 768, image
context only; config/wild-ir/models/modules/DenoisingUNet_arch.py, options/inference.yml:30-39)
and the ViT-L/14 DaCLIP encoder (model_configs/daclip_ViT-L-14.json). Fixtures: wild_*.npz /
wild_state_spec.json from make_golden.py gen_wild (the reference run here)."""
import json
import os

import numpy as np
import pytest
import torch

from daclip_amd import arch, synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def wild_images():
    return synth.synth_noise((1, 3, 224, 224), seed=41, tag="img4clip_wild")


def test_wild_state_spec_matches_reference():
    ref = json.load(open(os.path.join(GOLDEN, "wild_state_spec.json")))
    ours = arch.unet_state_spec(arch.WILD_IR_UNET)
    assert list(ref.items()) == [(k, list(v)) for k, v in ours.items()]


def test_oracle_wild_unet_matches_reference(golden):
    from oracle import unet as OU
    sd = synth.synth_state_dict(arch.unet_state_spec(arch.WILD_IR_UNET), 0)
    g = golden("wild_unet_fwd.npz")
    for tag in ("32x32", "48x40"):
        out = OU.forward(sd, g[tag + "_xt"], g[tag + "_mu"], 37.0, None, g[tag + "_ic"])
        assert rel(out, g[tag + "_out"]) < 2e-5


@pytest.mark.slow
def test_oracle_l14_encode_matches_reference(golden):
    from oracle import clip as OC
    sd = synth.synth_state_dict(arch.daclip_state_spec(arch.VIT_L_14, arch.TEXT_L_14), 0)
    ic, dc = OC.encode_image(sd, wild_images(), layers=24, heads=16)
    g = golden("wild_l14_encode.npz")
    assert rel(ic, g["image_context"]) < 1e-4 and rel(dc, g["degra_context"]) < 1e-4


@pytest.fixture(scope="module")
def wild_unets():
    from daclip_amd.unet import ConditionalUNet
    sd = synth.synth_state_dict(arch.unet_state_spec(arch.WILD_IR_UNET), 0)
    out = {}
    for dt in ("fp32", "bf16", "fp16"):
        m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 768, False, True, scale=0.5, dtype=dt)
        m.load_state_dict(sd)
        out[dt] = m
    return out


# Bars: fp32 exact-f32 MFMA; bf16 / fp16 storage with fp32 accumulation (fp16's 11-bit
# significand is 8x finer than bf16's: the bench's Wild-IR line runs fp16).
TOL = {"fp32": 1e-4, "bf16": 5e-2, "fp16": 1e-2}


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
def test_wild_unet_matches_reference(golden, wild_unets, dt):
    g = golden("wild_unet_fwd.npz")
    for tag in ("32x32", "48x40"):
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        out = wild_unets[dt](T(g[tag + "_xt"]), T(g[tag + "_mu"]), 37.0,
                             image_context=T(g[tag + "_ic"])).cpu().numpy()
        assert out.shape == g[tag + "_out"].shape
        r = rel(out, g[tag + "_out"])
        print(f"wild unet {dt} {tag}: rel {r:.3e}")
        assert r < TOL[dt]


@pytest.mark.gpu
def test_wild_loop_512_batch_invariant(wild_unets):
    """BASELINE config 4 resolution: a 512^2 posterior loop (3 steps, device noise) is finite
    and each image equals its single-image run (sharding across GPUs is bit-exact)."""
    from daclip_amd.sde import IRSDE
    m = wild_unets["bf16"]
    lq = torch.from_numpy(synth.synth_images(2, 512, 512, seed=71)).cuda()
    ic = torch.from_numpy(synth.synth_noise((2, 768), seed=72, tag="ic")).cuda()

    def run(lo, hi):
        s = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
        s.set_model(m)
        s.set_mu(lq[lo:hi])
        s.image_offset = lo
        return s.reverse_posterior(lq[lo:hi], T=3, image_context=ic[lo:hi])
    both = run(0, 2)
    assert torch.isfinite(both).all()
    assert torch.equal(both[1:], run(1, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
def test_l14_encode_matches_reference(golden, dt):
    from daclip_amd.open_clip import DaCLIP
    m = DaCLIP(arch.VIT_L_14, arch.TEXT_L_14, dtype=dt, with_text=False)
    m.load_synthetic(0)
    ic, dc = m.encode_image(torch.from_numpy(wild_images()).cuda(), control=True)
    g = golden("wild_l14_encode.npz")
    ri, rd = rel(ic.cpu().numpy(), g["image_context"]), rel(dc.cpu().numpy(), g["degra_context"])
    print(f"l14 encode {dt}: rel image {ri:.3e} degra {rd:.3e}")
    assert ri < TOL[dt] and rd < TOL[dt]
