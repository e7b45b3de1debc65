"""The state_dict layouts in daclip_amd.arch equal the reference modules' (state_spec.json)."""
import json
import os

from conftest import GOLDEN
from daclip_amd import arch


def _ref(name):
    spec = json.load(open(os.path.join(GOLDEN, "state_spec.json")))[name]
    return [(k, tuple(s)) for k, s in spec]


def test_unet_spec_nf64():
    assert list(arch.unet_state_spec(arch.UNetConfig()).items()) == _ref("unet_nf64")


def test_unet_spec_nf32():
    assert list(arch.unet_state_spec(arch.UNetConfig(nf=32)).items()) == _ref("unet_nf32")


def test_daclip_spec_b32():
    ours = arch.daclip_state_spec(arch.VIT_B_32, arch.TEXT_B_32)
    assert sorted(ours.items()) == sorted(_ref("daclip_b32"))
    assert len(ours) == 631


def test_reference_flop_model_reproduces_survey_constants():
    """the reference's work per step / encode, from shapes (torch flop_counter
    convention on the reference's CPU path), to the precision the survey quotes."""
    from daclip_amd import arch
    gf = lambda f: f / 1e9
    assert round(gf(arch.reference_unet_flops(arch.UNetConfig(), 256, 256)), 3) == 266.172
    assert round(gf(arch.reference_unet_flops(arch.UNetConfig(), 512, 512)), 2) == 1129.09
    assert round(gf(arch.reference_unet_flops(arch.WILD_IR_UNET, 512, 512)), 2) == 348.88
    assert round(gf(arch.reference_encode_flops(arch.VIT_B_32)), 3) == 18.159
    assert round(gf(arch.reference_encode_flops(arch.VIT_L_14)), 1) == 324.0
    assert round(arch.reference_tflop_per_image(arch.UNetConfig(), arch.VIT_B_32, 256, 256, 100), 3) == 26.635
