"""The SpatialTransformer / LinearAttention norm folds in the network (engine.cpp sptrans /
linattn): the norm1 LayerNorm folded into q|k|v, the GroupNorm applied in proj_in's A path with
its statistics from the PreNorm LayerNorm, and the C = 256 LinearAttention PreNorm folded into
to_qkv (attention.py:76-77, 239-261; module_util.py:77-97, 157-185). One bf16 256x256 forward
(every folded shape at the 32x32 / 64x64 levels) with the folds on (the default DAC_FOLD mask)
and off (DAC_FOLD=0, read when the handle packs its weights and per forward), each against the
fp32 numpy oracle: the folded path must be as close to the oracle as
the unfolded one (bound 1.5e-2 max-rel, the bf16 forward bar of test_hip_parity.py), and the two
bf16 outputs must agree to bf16 noise."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def _forward(unet_sd, fold, x, mu, tc, ic):
    from daclip_amd.unet import ConditionalUNet
    old = {k: os.environ.get(k) for k in ("DAC_FOLD",)}
    if fold:
        os.environ.pop("DAC_FOLD", None)
    else:
        os.environ["DAC_FOLD"] = "0"
    try:
        m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype="bf16")
        m.load_state_dict(unet_sd)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        return m(T(x), T(mu), 77.0, text_context=T(tc), image_context=T(ic)).cpu().numpy()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_norm_folds_match_unfolded_and_oracle(unet_sd):
    from daclip_amd import synth
    from oracle import unet as OU
    x = synth.synth_noise((1, 3, 256, 256), seed=41, tag="x256") * 0.3 + 0.5
    mu = synth.synth_images(1, 256, 256, seed=42)
    tc = synth.synth_noise((1, 512), seed=43, tag="tc") * 0.5
    ic = synth.synth_noise((1, 512), seed=44, tag="ic") * 0.5
    ref = OU.forward(unet_sd, x, mu, 77.0, tc, ic)
    on = _forward(unet_sd, True, x, mu, tc, ic)
    off = _forward(unet_sd, False, x, mu, tc, ic)
    e_on, e_off, d = rel(on, ref), rel(off, ref), rel(on, off)
    print(f"bf16 256 forward vs oracle: folded {e_on:.3e}, unfolded {e_off:.3e}; folded vs unfolded {d:.3e}")
    assert np.isfinite(on).all()
    assert e_on < 1.5e-2 and e_on < 1.5 * e_off + 1e-3
    assert d < 1.5e-2
