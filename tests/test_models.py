"""create_model / DenoisingModel / Predictor mirrors (daclip_amd/models.py, predict.py)."""
import os

import numpy as np
import pytest
import torch

from daclip_amd import models

OPT = {
    "model": "denoising",
    "sde": {"max_sigma": 50, "T": 100, "schedule": "cosine", "eps": 0.005, "sampling_mode": "posterior"},
    "network_G": {"which_model_G": "ConditionalUNet",
                  "setting": {"in_nc": 3, "out_nc": 3, "nf": 64, "ch_mult": [1, 2, 4, 8],
                              "context_dim": 512, "use_degra_context": True, "use_image_context": True}},
    "path": {"pretrain_model_G": None, "daclip": None},
}


def test_clean_state_dict_strips_module_prefix():
    sd = {"module.a.weight": 1, "b.bias": 2, "module.module.c": 3}
    out = models.clean_state_dict(sd)
    assert list(out) == ["a.weight", "b.bias", "module.c"]


def test_parse_options_roundtrip(tmp_path):
    import yaml
    p = tmp_path / "test.yml"
    p.write_text(yaml.safe_dump(OPT))
    assert models.parse_options(str(p)) == OPT


def test_create_model_rejects_unknown():
    with pytest.raises(NotImplementedError):
        models.create_model(dict(OPT, model="sr"))
    bad = dict(OPT, network_G={"which_model_G": "UNet", "setting": {}})
    with pytest.raises(NotImplementedError):
        models.DenoisingModel(bad)


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_no_gpu_fails_loudly():
    with pytest.raises((RuntimeError, ImportError)):
        models.create_model(OPT)


@pytest.mark.gpu
def test_checkpoint_roundtrip_module_prefix(tmp_path, unet_sd):
    """A DataParallel-style checkpoint (module.* keys) loads through opt.path.pretrain_model_G
    (torch.load weights_only) and gives the same forward as a direct load."""
    ck = tmp_path / "universal-ir.pth"
    torch.save({"module." + k: torch.from_numpy(v) for k, v in unet_sd.items()}, ck)
    opt = dict(OPT, path={"pretrain_model_G": str(ck), "strict_load": True})
    m = models.create_model(opt)
    from daclip_amd.unet import ConditionalUNet
    ref = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True)
    ref.load_state_dict(unet_sd)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 3, 32, 32, generator=g).cuda()
    mu = torch.rand(1, 3, 32, 32, generator=g).cuda()
    c = torch.randn(1, 512, generator=g).cuda()
    a = m.model(x, mu, 10.0, text_context=c, image_context=c)
    b = ref(x, mu, 10.0, text_context=c, image_context=c)
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_predictor_batch_matches_manual_pipeline():
    """Predictor.predict_batch == the predict.py op sequence written out by hand."""
    from daclip_amd.predict import Predictor
    from daclip_amd.preprocess import clip_transform, tensor2img
    from daclip_amd import synth
    opt = dict(OPT, sde=dict(OPT["sde"], T=5))
    p = Predictor()
    p.setup(opt, synthetic=True)
    imgs = [(synth.synth_images(1, 40, 48, seed=s)[0].transpose(1, 2, 0)[:, :, ::-1] * 255).round()
            .astype(np.uint8) for s in (1, 2)]
    seed0 = p.sde.seed
    torch.manual_seed(123)
    out = p.predict_batch(imgs)
    assert len(out) == 2 and out[0].shape == (40, 48, 3) and out[0].dtype == np.uint8
    torch.manual_seed(123)
    rgb = [im[:, :, [2, 1, 0]] / 255.0 for im in imgs]
    ic, dc = p.clip_model.encode_image(torch.stack([clip_transform(r) for r in rgb]).cuda(), control=True)
    lq = torch.stack([torch.tensor(r, dtype=torch.float32).permute(2, 0, 1) for r in rgb])
    noisy = p.sde.noise_state(lq)
    p.sde.set_mu(lq.cuda())
    p.sde.seed = seed0                      # same device-noise stream as the first call
    res = p.sde.reverse_posterior(noisy.cuda(), text_context=dc.float(), image_context=ic.float())
    for i in range(2):
        assert np.array_equal(out[i], tensor2img(res[i].cpu()))


def test_make_grid_matches_torchvision_layout():
    from daclip_amd.preprocess import make_grid
    t = torch.arange(3 * 2 * 2 * 3, dtype=torch.float32).reshape(3, 2, 2, 3)
    t = torch.cat([t, t[:, :1]], 1)                      # 3 channels
    g = make_grid(t, nrow=2, padding=1)
    assert g.shape == (3, 2 * 3 + 1, 2 * 4 + 1)
    assert torch.equal(g[:, 1:3, 1:4], t[0]) and torch.equal(g[:, 1:3, 5:8], t[1])
    assert torch.equal(g[:, 4:6, 1:4], t[2]) and float(g[:, 4:6, 5:8].abs().sum()) == 0.0
    assert torch.equal(make_grid(t[:1]), t[0])


@pytest.mark.gpu
def test_save_states_semantics(tmp_path):
    """sde_utils.py:305-311: a state PNG every T//100 steps (channel halves side by side);
    3-channel states fail in torch.cat like the reference; T < 100 -> interval 0 raises."""
    from daclip_amd.sde import IRSDE
    from PIL import Image
    s = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    x6 = torch.rand(1, 6, 8, 8, device="cuda")
    s.set_mu(torch.rand(1, 6, 8, 8, device="cuda"))
    s.set_model(lambda x, mu, t, **k: 0.1 * (x - mu))
    s.reverse_posterior(x6, T=3, save_states=True, save_dir=str(tmp_path / "st"))
    files = sorted(p.name for p in (tmp_path / "st").iterdir())
    assert files == ["state_1.png", "state_2.png", "state_3.png"]
    assert Image.open(tmp_path / "st" / "state_1.png").size == (16, 8)
    s.set_mu(torch.rand(1, 3, 8, 8, device="cuda"))
    with pytest.raises(RuntimeError):
        s.reverse_posterior(torch.rand(1, 3, 8, 8, device="cuda"), T=2, save_states=True,
                            save_dir=str(tmp_path / "st3"))
    s10 = IRSDE(max_sigma=50, T=10, schedule="cosine", eps=0.005)
    s10.set_mu(torch.rand(1, 6, 8, 8, device="cuda"))
    s10.set_model(lambda x, mu, t, **k: 0.1 * x)
    with pytest.raises(ZeroDivisionError):
        s10.reverse_posterior(x6, T=2, save_states=True, save_dir=str(tmp_path / "s10"))
