"""Evaluation-side host code (§8f rank 4): metrics (utils/img_utils.py:182-234,
data/util.py:189-210), the LQGT folder dataset (data/LQGT_dataset.py) and the test.py-style
batch evaluation."""
import numpy as np
import pytest
import torch
from PIL import Image

from daclip_amd import metrics


def test_bgr2ycbcr_matches_reference(golden):
    g = golden("img_metrics.npz")
    ua = g["ua"]
    assert np.array_equal(metrics.bgr2ycbcr(ua, True), g["y_u8"])
    assert np.array_equal(metrics.bgr2ycbcr(ua, False), g["ycc_u8"])
    fa = ua.astype(np.float64) / 255.0
    np.testing.assert_allclose(metrics.bgr2ycbcr(fa, True), g["y_f"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(metrics.bgr2ycbcr(fa, False), g["ycc_f"], rtol=0, atol=1e-12)
    before = fa.copy()
    metrics.bgr2ycbcr(fa, True)
    assert np.array_equal(fa, before)                   # no in-place scaling of the input


def _ssim_direct(a, b):
    """Independent restatement: explicit 11x11 window sums at every valid position."""
    a, b = a.astype(np.float64), b.astype(np.float64)
    w = metrics.gaussian_window()
    c1, c2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    H, W = a.shape[:2]
    vals = []
    for i in range(H - 10):
        for j in range(W - 10):
            pa, pb = a[i:i + 11, j:j + 11], b[i:i + 11, j:j + 11]
            ww = w if a.ndim == 2 else w[:, :, None]
            m1, m2 = (pa * ww).sum((0, 1)), (pb * ww).sum((0, 1))
            s1 = (pa * pa * ww).sum((0, 1)) - m1 * m1
            s2 = (pb * pb * ww).sum((0, 1)) - m2 * m2
            s12 = (pa * pb * ww).sum((0, 1)) - m1 * m2
            vals.append(((2 * m1 * m2 + c1) * (2 * s12 + c2)) / ((m1 * m1 + m2 * m2 + c1) * (s1 + s2 + c2)))
    return float(np.mean(vals))


def test_ssim_properties(golden):
    g = golden("img_metrics.npz")
    ua, ub = g["ua"], g["ub"]
    assert metrics.calculate_ssim(ua, ua) == pytest.approx(1.0, abs=1e-12)
    s = metrics.calculate_ssim(ua, ub)
    assert 0.0 < s < 1.0 and s == pytest.approx(metrics.calculate_ssim(ub, ua), abs=1e-12)
    assert s == pytest.approx(_ssim_direct(ua, ub), abs=1e-10)
    y = metrics.bgr2ycbcr(ua, True)
    assert metrics.calculate_ssim(y, metrics.bgr2ycbcr(ub, True)) == pytest.approx(
        _ssim_direct(y, metrics.bgr2ycbcr(ub, True)), abs=1e-10)
    assert metrics.gaussian_window().sum() == pytest.approx(1.0)
    with pytest.raises(ValueError):
        metrics.calculate_ssim(ua, ua[:-1])


def test_psnr_matches_reference(golden):
    g = golden("img_metrics.npz")
    assert metrics.calculate_psnr(g["ua"], g["ub"]) == pytest.approx(float(g["psnr"]), abs=1e-12)
    assert metrics.calculate_psnr(g["ua"], g["ua"]) == float("inf")


def _write_pair(root, n=3, sizes=((32, 32), (32, 32), (40, 48))):
    lq, gt = root / "LQ", root / "GT"
    lq.mkdir(), gt.mkdir()
    rng = np.random.default_rng(0)
    for i in range(n):
        h, w = sizes[i]
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(a).save(lq / f"img{i}.png")
        Image.fromarray(np.clip(a.astype(int) + 7, 0, 255).astype(np.uint8)).save(gt / f"img{i}.png")
    return str(lq), str(gt)


def test_lqgt_dataset_layout(tmp_path):
    from daclip_amd.data import LQGTDataset, read_img
    lq, gt = _write_pair(tmp_path)
    ds = LQGTDataset(lq, gt)
    assert len(ds) == 3
    it = ds[0]
    assert it["LQ"].shape == (3, 32, 32) and it["GT"].shape == (3, 32, 32) and it["LQ_clip"].shape == (3, 224, 224)
    rgb = np.asarray(Image.open(it["LQ_path"])).astype(np.float32) / 255.0
    assert np.array_equal(it["LQ"].numpy(), rgb.transpose(2, 0, 1))        # RGB CHW, like the reference
    assert np.array_equal(read_img(it["LQ_path"]), rgb[:, :, ::-1])          # cv2 layout: BGR
    Image.fromarray(np.zeros((8, 8), np.uint8)).save(tmp_path / "g.png")
    assert read_img(str(tmp_path / "g.png")).shape == (8, 8, 1)
    (tmp_path / "empty").mkdir()
    with pytest.raises(RuntimeError):
        LQGTDataset(str(tmp_path / "empty"))


@pytest.mark.gpu
def test_evaluate_folder(tmp_path):
    from daclip_amd.evaluate import evaluate
    opt = {"model": "denoising",
           "sde": {"max_sigma": 50, "T": 3, "schedule": "cosine", "eps": 0.005, "sampling_mode": "posterior"},
           "network_G": {"which_model_G": "ConditionalUNet",
                         "setting": {"in_nc": 3, "out_nc": 3, "nf": 64, "ch_mult": [1, 2, 4, 8],
                                     "context_dim": 512, "use_degra_context": True, "use_image_context": True}},
           "path": {"pretrain_model_G": None}}
    lq, gt = _write_pair(tmp_path)
    res = evaluate(opt, lq, gt, str(tmp_path / "out"), batch=2, synthetic=True)
    assert res["summary"]["images"] == 3
    assert sorted(p.name for p in (tmp_path / "out").iterdir()) == ["img0.png", "img1.png", "img2.png"]
    for k in ("psnr", "ssim", "psnr_y", "ssim_y"):
        assert np.isfinite(res["summary"][k])
    assert Image.open(tmp_path / "out" / "img2.png").size == (48, 40)


def test_evaluate_crop_border_follows_test_py():
    """config/daclip-sde/test.py:84, 150: crop_border = opt["crop_border"] if set, else
    opt["degradation"]["scale"] (4 in options/test.yml:20); an explicit argument wins."""
    from daclip_amd.evaluate import resolve_crop_border
    opt = {"degradation": {"sigma": 25, "noise_type": "G", "scale": 4}}
    assert resolve_crop_border(opt) == 4
    assert resolve_crop_border(dict(opt, crop_border=None)) == 4
    assert resolve_crop_border(dict(opt, crop_border=0)) == 4            # falsy -> scale, as test.py
    assert resolve_crop_border(dict(opt, crop_border=2)) == 2
    assert resolve_crop_border(opt, 0) == 0
    assert resolve_crop_border({}) == 0
