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
