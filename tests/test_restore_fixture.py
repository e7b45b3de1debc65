"""The restoration fixture (tests/golden/restore_rain_256_t100.npz, made by running the
reference's predict.py:58-91 flow on the 256x256 centre crop of images/3_rain.png with the
tracking weights of synth.tracking_state_dict; make_golden.py gen_restore) is not degenerate,
and the oracle reproduces the reference on it. CPU only: the oracle restates the last
posterior step (sde_utils.py:227-231, 245-247) from the state the reference's loop reached,
and the last reverse_sde step (sde_utils.py:44-45, 177-187) of the 64x64 run."""
import numpy as np

from oracle import sde as OS, unet as OU, imgs as OI


def test_fixture_is_in_range_and_nontrivial(restore_fixture):
    g, _, _ = restore_fixture
    out = g["out"]
    inr = float(((out > 0) & (out < 1)).mean())
    assert inr >= 0.90, inr                         # >= 90 % of pixels in (0, 1)
    assert np.abs(out).max() < 1.5
    psnr = float(g["psnr_out_vs_lq"])
    assert 20.0 < psnr < 40.0, psnr                 # restores away from the LQ, stays an image
    assert float(((g["out_sde64"] > 0) & (g["out_sde64"] < 1)).mean()) >= 0.90
    assert float(g["fit_rel"]) < 1e-3               # fitted scales track g1, g2 within 0.1 %
    assert OI.calculate_psnr(g["out_u8"], g["lq_u8"]) == psnr


def test_fixture_lq_is_the_rain_crop(restore_fixture):
    g, _, _ = restore_fixture
    assert g["rgb_u8"].shape == (256, 256, 3) and g["rgb_u8"].dtype == np.uint8
    lq = g["rgb_u8"].astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    assert np.array_equal(OI.tensor2img(lq), g["lq_u8"])


def test_oracle_last_posterior_step_matches_reference(restore_fixture):
    g, sd, noise = restore_fixture
    lq = (g["rgb_u8"] / 255.0).astype(np.float32).transpose(2, 0, 1)[None]
    s = OS.IRSDE(50, 100, "cosine", 0.005)
    s.mu = lq
    eps = OU.forward(sd, g["x_t1"], lq, 1.0, g["degra_context"], g["image_context"])
    out = s.posterior_step(g["x_t1"], eps, 1, noise["steps"][99])
    err = np.abs(out - g["out"]).max()
    assert err < 1e-4, err                          # fp32 summation order (0.03 levels)
    u8 = OI.tensor2img(out[0]).astype(int)
    assert np.abs(u8 - g["out_u8"]).max() <= 1     # rounding ties only
    assert np.mean(u8 != g["out_u8"]) < 1e-3


def test_oracle_last_sde_step_matches_reference(restore_fixture):
    g, sd, noise = restore_fixture
    lq = (g["rgb_u8"] / 255.0).astype(np.float32).transpose(2, 0, 1)[None][:, :, 96:160, 96:160]
    s = OS.IRSDE(50, 100, "cosine", 0.005)
    s.mu = np.ascontiguousarray(lq)
    eps = OU.forward(sd, g["x_t1_sde64"], s.mu, 1.0, g["degra_context"], g["image_context"])
    out = s.sde_step(g["x_t1_sde64"], eps, 1, noise["steps_64"][99])
    err = np.abs(out - g["out_sde64"]).max()
    assert err < 1e-4, err                          # fp32 summation order
