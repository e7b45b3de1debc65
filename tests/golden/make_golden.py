"""Generate the committed golden fixtures by running the REFERENCE on CPU, in this container.

    cd tests/golden && python make_golden.py

Only the outputs (.npz / .json under tests/golden/) are committed; the reference itself
never leaves this container. Weights are deterministic synthetic tensors from
daclip_amd.synth (no released checkpoint exists offline), loaded into the reference
modules with strict load_state_dict. Random draws inside the reference sampler
(torch.randn_like in sde_utils.py:184, 231, 375) are replaced by injected, pre-generated
noise so the oracle and the HIP path can consume the identical tensors.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "da-clip_amd"))

import _refimport  # noqa: E402
from daclip_amd import synth  # noqa: E402

torch.set_grad_enabled(False)
torch.set_num_threads(8)
ConditionalUNet, open_clip, ref_utils = _refimport.import_reference()
from open_clip.model import CLIP  # noqa: E402
from open_clip.daclip_model import DaCLIP  # noqa: E402


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def load(model, seed=0):
    sd = model.state_dict()
    spec = {k: tuple(v.shape) for k, v in sd.items()}
    w = synth.synth_state_dict(spec, seed)
    model.load_state_dict({k: T(v) for k, v in w.items()}, strict=True)
    return spec


class NoiseInjector:
    """Replaces torch.randn_like with a queue of pre-generated tensors."""

    def __init__(self, noises):
        self.q = list(noises)
        self.orig = torch.randn_like

    def __enter__(self):
        def fake(x, *a, **k):
            n = self.q.pop(0)
            assert tuple(n.shape) == tuple(x.shape), (n.shape, x.shape)
            return T(n).to(x.dtype)
        torch.randn_like = fake
        return self

    def __exit__(self, *exc):
        torch.randn_like = self.orig
        assert not self.q, f"{len(self.q)} injected noises unused"


def unet_cfg(nf=64):
    return dict(in_nc=3, out_nc=3, nf=nf, ch_mult=[1, 2, 4, 8], context_dim=512,
                use_degra_context=True, use_image_context=True)


def gen_state_spec():
    m = ConditionalUNet(**unet_cfg(64))
    spec = {"unet_nf64": [[k, list(v.shape)] for k, v in m.state_dict().items()]}
    m32 = ConditionalUNet(**unet_cfg(32))
    spec["unet_nf32"] = [[k, list(v.shape)] for k, v in m32.state_dict().items()]
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    cfg.pop("custom_text")
    d = DaCLIP(CLIP(**cfg))
    spec["daclip_b32"] = [[k, list(v.shape)] for k, v in d.state_dict().items()]
    with open(os.path.join(HERE, "state_spec.json"), "w") as f:
        json.dump(spec, f)


def gen_unet_forward():
    m = ConditionalUNet(**unet_cfg(64)).eval()
    load(m, seed=0)
    for (b, h, w, t, tag) in [(2, 32, 32, 57.0, "32x32"), (1, 30, 34, 3.0, "30x34"),
                              (1, 64, 64, 100.0, "64x64")]:
        xt = synth.synth_noise((b, 3, h, w), seed=1, tag="xt" + tag) * 0.3 + 0.5
        mu = synth.synth_images(b, h, w, seed=2)
        tc = synth.synth_noise((b, 512), seed=3, tag="text") * 0.5
        ic = synth.synth_noise((b, 512), seed=4, tag="image") * 0.5
        out = m(T(xt), T(mu), t, text_context=T(tc), image_context=T(ic)).numpy()
        np.savez_compressed(os.path.join(HERE, f"unet_fwd_nf64_{tag}.npz"), xt=xt, mu=mu,
                            t=np.float32(t), text_context=tc, image_context=ic, out=out)


def gen_sde():
    sde = ref_utils.IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005, device="cpu")
    lin = ref_utils.IRSDE(max_sigma=50, T=100, schedule="linear", eps=0.005, device="cpu")
    tabs = {}
    for name, s in (("cos", sde), ("lin", lin)):
        for f in ("thetas", "sigmas", "thetas_cumsum", "sigma_bars"):
            tabs[f"{name}_{f}"] = getattr(s, f).numpy()
        tabs[f"{name}_dt"] = np.float32(s.dt.item())
    tabs["max_sigma"] = np.float32(sde.max_sigma)
    np.savez_compressed(os.path.join(HERE, "sde_tables.npz"), **tabs)

    # Full T=100 posterior loop + a 3-step reverse_sde, UNet nf=64 at 16x16, B=1.
    m = ConditionalUNet(**unet_cfg(64)).eval()
    load(m, seed=0)
    sde.set_model(m)
    b, h, w = 1, 16, 16
    lq = synth.synth_images(b, h, w, seed=7)
    tc = synth.synth_noise((b, 512), seed=3, tag="text") * 0.5
    ic = synth.synth_noise((b, 512), seed=4, tag="image") * 0.5
    n0 = synth.synth_noise((b, 3, h, w), seed=8, tag="noise_state")
    steps = synth.synth_noise((100, b, 3, h, w), seed=9, tag="steps")
    with NoiseInjector([n0]):
        noisy = sde.noise_state(T(lq))
    sde.set_mu(T(lq))
    with NoiseInjector(list(steps)):
        out = sde.reverse_posterior(noisy, text_context=T(tc), image_context=T(ic)).numpy()
    with NoiseInjector(list(steps[:3])):
        out_sde = sde.reverse_sde(noisy, T=3, text_context=T(tc), image_context=T(ic)).numpy()
    out_u8 = ref_utils.tensor2img(T(out.copy()).squeeze())
    lq_u8 = ref_utils.tensor2img(T(lq.copy()).squeeze())
    psnr = ref_utils.calculate_psnr(out_u8, lq_u8)
    np.savez_compressed(os.path.join(HERE, "posterior_loop_16x16.npz"), lq=lq, text_context=tc,
                        image_context=ic, noise_state=n0, step_noise=steps, noisy=noisy.numpy(),
                        out=out, out_sde3=out_sde, out_u8=out_u8, lq_u8=lq_u8,
                        psnr=np.float64(psnr))


HEADLINE_IMAGE = "/root/reference/images/00006.jpg"      # a real 256x256 LQ photo
HEADLINE_T = 100


def headline_noise(shape_lq):
    """Injected noises of the headline fixture (regenerated by the tests, never stored):
    noise_state draw [1,3,H,W] and the T per-step draws [T,1,3,H,W]."""
    n0 = synth.synth_noise(shape_lq, seed=71, tag="hl_noise_state")
    steps = synth.synth_noise((HEADLINE_T,) + tuple(shape_lq), seed=72, tag="hl_steps")
    return n0, steps


def gen_headline():
    """The benchmarked configuration pinned end to end on a real image (predict.py:58-91):
    PIL-decoded 256x256 RGB -> /255 (float64, as predict.py:64) -> clip_transform (PIL
    restatement, daclip_amd.preprocess; torchvision is absent) -> reference DaCLIP ViT-B/32
    encode_image(control=True) -> reference noise_state + T=100 reverse_posterior of the
    reference ConditionalUNet (nf=64) with injected noise -> tensor2img. Synthetic seeded
    weights (seed 0) for both networks; fp32 CPU, i.e. the reference CPU path."""
    from PIL import Image
    from daclip_amd.preprocess import clip_transform
    rgb = np.asarray(Image.open(HEADLINE_IMAGE).convert("RGB"))
    image = rgb / 255.0                                              # predict.py:64 (float64)
    img4clip = clip_transform(image).unsqueeze(0).numpy()
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    ic, dc = d.encode_image(T(img4clip), control=True)
    ic, dc = ic.float(), dc.float()
    lq = torch.tensor(image, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0)   # predict.py:73-75
    m = ConditionalUNet(**unet_cfg(64)).eval()
    load(m, seed=0)
    sde = ref_utils.IRSDE(max_sigma=50, T=HEADLINE_T, schedule="cosine", eps=0.005, device="cpu")
    sde.set_model(m)
    n0, steps = headline_noise(tuple(lq.shape))
    with NoiseInjector([n0]):
        noisy = sde.noise_state(lq)
    sde.set_mu(lq)
    with NoiseInjector(list(steps)):
        out = sde.reverse_posterior(noisy, text_context=dc, image_context=ic).numpy()
    out_u8 = ref_utils.tensor2img(T(out.copy()).squeeze())
    lq_u8 = ref_utils.tensor2img(lq.squeeze())
    np.savez_compressed(os.path.join(HERE, "headline_256_t100.npz"), rgb_u8=rgb, img4clip=img4clip,
                        image_context=ic.numpy(), degra_context=dc.numpy(), out=out, out_u8=out_u8,
                        lq_u8=lq_u8, psnr_out_vs_lq=np.float64(ref_utils.calculate_psnr(out_u8, lq_u8)))


RESTORE_IMAGE = "/root/reference/images/3_rain.png"     # BASELINE configs[0]: the rainy sample
RESTORE_T = synth.TRACK_T


def restore_noise(shape_lq, T=RESTORE_T, tag="rs"):
    """Injected noises of the restoration fixtures (regenerated by the tests, never stored)."""
    n0 = synth.synth_noise(shape_lq, seed=91, tag=tag + "_noise_state")
    steps = synth.synth_noise((T,) + tuple(shape_lq), seed=92, tag=tag + "_steps")
    return n0, steps


def rain_crop():
    """256x256 centre crop of the rainy sample (720x480), uint8 RGB."""
    from PIL import Image
    im = np.asarray(Image.open(RESTORE_IMAGE).convert("RGB"))
    h, w = im.shape[:2]
    y, x = (h - 256) // 2, (w - 256) // 2
    return np.ascontiguousarray(im[y:y + 256, x:x + 256])


def fit_tracking(base, sde, features, deep_calib):
    """Fits synth.tracking_state_dict's free parameters on the reference modules: the
    final_res_block scale rows (exact triangular solve on the reference's own hinge features
    SiLU(t_emb(t)), t = 1..T; the hinges decrease in t, so the sums carry no cancellation) and
    k, which scales D to std 0.04 on the fixture image at t = 1."""
    kd = synth.TRACK_KNOTS
    z = np.zeros(len(kd), np.float32)
    sd0 = synth.tracking_state_dict(base, z, z, 1.0)
    F = features(sd0).astype(np.float64)[:, kd]
    tt = np.arange(1, RESTORE_T + 1)
    sbar = sde.sigma_bars.numpy()[tt].astype(np.float64)
    ea = np.exp(sde.thetas_cumsum.numpy()[tt].astype(np.float64) * float(sde.dt))
    g1, g2 = 1.0 / sbar, 1.0 / (sbar * ea)
    w1 = np.linalg.solve(F, g1 - 1.0).astype(np.float32)
    w2 = np.linalg.solve(F, g2 - 1.0).astype(np.float32)
    A = synth.tracking_projection().astype(np.float64)
    xin = deep_calib(sd0)[:, :64].astype(np.float64)
    D = torch.nn.functional.conv2d(T(xin), T(A), padding=1).numpy()
    k = float(np.float32(0.04 / D.std()))
    return synth.tracking_state_dict(base, w1, w2, k), dict(g1=g1, g2=g2, w1=w1, w2=w2, k=k)


def gen_restore():
    """A restoration fixture on which the PSNR bar means something: the
    reference's predict.py:58-91 flow on the 256x256 centre crop of images/3_rain.png
    (BASELINE configs[0]) with synth.tracking_state_dict UNet weights (seed-0 synthetic weights
    plus the fitted scale rows w_g1 / w_g2 and k, stored in the fixture), seed-0 ViT-B/32 DaCLIP, injected
    noise, T=100 posterior, fp32 CPU; plus a full T=100 reverse_sde run at 64x64 with the same
    weights (sde_utils.py:261-277)."""
    from daclip_amd.preprocess import clip_transform
    rgb = rain_crop()
    image = rgb / 255.0                                              # predict.py:64 (float64)
    img4clip = clip_transform(image).unsqueeze(0).numpy()
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    ic, dc = d.encode_image(T(img4clip), control=True)
    ic, dc = ic.float(), dc.float()
    lq = torch.tensor(image, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0)   # predict.py:73-75
    m = ConditionalUNet(**unet_cfg(64)).eval()
    spec = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    base = synth.synth_state_dict(spec, 0)
    sde = ref_utils.IRSDE(max_sigma=50, T=RESTORE_T, schedule="cosine", eps=0.005, device="cpu")

    def set_sd(sd):
        m.load_state_dict({k: T(v) for k, v in sd.items()}, strict=True)

    def features(sd):
        set_sd(sd)
        return np.concatenate([torch.nn.functional.silu(m.time_mlp(torch.tensor([float(t)]))).numpy()
                               for t in range(1, RESTORE_T + 1)])

    def deep_calib(sd):
        set_sd(sd)
        grab = {}
        hk = m.final_res_block.register_forward_hook(lambda mod, a, o: grab.update(x=a[0]))
        xt = lq + 0.004 * torch.from_numpy(synth.synth_noise(tuple(lq.shape), seed=93, tag="calib"))
        m(xt, lq, 1.0, text_context=dc, image_context=ic)
        hk.remove()
        return grab["x"].numpy()

    sd, info = fit_tracking(base, sde, features, deep_calib)
    set_sd(sd)
    # the fitted scales as the reference computes them
    ss = np.concatenate([m.final_res_block.mlp(m.time_mlp(torch.tensor([float(t)]))).numpy()
                         for t in range(1, RESTORE_T + 1)])
    fit1 = np.abs((ss[:, 0] + 1) / info["g1"] - 1).max()
    fit2 = np.abs((ss[:, 6] + 1) / info["g2"] - 1).max()
    print(f"fit rel err g1 {fit1:.2e} g2 {fit2:.2e} k {info['k']:.4g}", flush=True)
    seen = {}

    def model(x, mu, t, **kw):                 # records the state the last step starts from
        if float(t) == 1.0:
            seen[tuple(x.shape)] = x.clone().numpy()
        return m(x, mu, t, **kw)
    sde.set_model(model)
    n0, steps = restore_noise(tuple(lq.shape))
    with NoiseInjector([n0]):
        noisy = sde.noise_state(lq)
    sde.set_mu(lq)
    with NoiseInjector(list(steps)):
        out = sde.reverse_posterior(noisy, text_context=dc, image_context=ic).numpy()
    out_u8 = ref_utils.tensor2img(T(out.copy()).squeeze())
    lq_u8 = ref_utils.tensor2img(lq.squeeze())
    inr = float(((out > 0) & (out < 1)).mean())
    psnr = ref_utils.calculate_psnr(out_u8, lq_u8)
    Dl = 255 * (out[0].astype(np.float64) - lq[0].numpy())
    print(f"restore: in-range {inr:.4f} range [{out.min():.3f},{out.max():.3f}] psnr vs lq {psnr:.3f} "
          f"D/level mean {Dl.mean(axis=(1, 2))} std {Dl.std(axis=(1, 2))} "
          f"frac hist {np.histogram(Dl - np.round(Dl), bins=10)[0]}", flush=True)
    # full-length reverse_sde at 64x64 (a crop of the same image), same weights and contexts
    lq64 = lq[:, :, 96:160, 96:160].contiguous()
    s0, ssteps = restore_noise(tuple(lq64.shape), tag="sde64")
    sde.set_mu(lq64)
    with NoiseInjector([s0]):
        noisy64 = sde.noise_state(lq64)
    with NoiseInjector(list(ssteps)):
        out_sde = sde.reverse_sde(noisy64, text_context=dc, image_context=ic).numpy()
    print(f"sde64: in-range {float(((out_sde > 0) & (out_sde < 1)).mean()):.4f} "
          f"range [{out_sde.min():.3f},{out_sde.max():.3f}]", flush=True)
    np.savez_compressed(os.path.join(HERE, "restore_rain_256_t100.npz"), rgb_u8=rgb, img4clip=img4clip,
                        image_context=ic.numpy(), degra_context=dc.numpy(), out=out, out_u8=out_u8,
                        lq_u8=lq_u8, psnr_out_vs_lq=np.float64(psnr), out_sde64=out_sde,
                        fit_rel=np.float64(max(fit1, fit2)), w_g1=info["w1"], w_g2=info["w2"],
                        k=np.float32(info["k"]), x_t1=seen[tuple(lq.shape)],
                        x_t1_sde64=seen[tuple(lq64.shape)])


# BASELINE configs[2]'s per-GPU slice: 8 distinct real LQ photos of the reference's sample set,
# chosen across options/test.yml:4's degradation classes by their source datasets (file names):
MIXED_IMAGES = ["3_rain.png",                 # rainy (Rain100H-style sample, BASELINE configs[0])
                "0048_0.9_0.2.jpg",           # hazy (RESIDE naming: id_A_beta)
                "GOPR0871_11_00_000078.png",  # motion-blurry (GoPro)
                "179.png",                    # low-light (LOL, 600x400)
                "21077.png",                  # BSD-size (481x321): noisy / jpeg-compressed sets
                "IMG_6444.jpg",               # raindrop-style capture
                "sailing2.png",               # shadowed / inpainting sample
                "beautiful_smile_00489.jpg"]  # face (snowy / uncompleted samples are faces too)
MIXED_T = synth.TRACK_T


def mixed_crops():
    """uint8 RGB [8,256,256,3]: the 256x256 centre crop of each MIXED_IMAGES photo."""
    from PIL import Image
    out = []
    for f in MIXED_IMAGES:
        im = np.asarray(Image.open("/root/reference/images/" + f).convert("RGB"))
        h, w = im.shape[:2]
        y, x = (h - 256) // 2, (w - 256) // 2
        out.append(im[y:y + 256, x:x + 256])
    return np.ascontiguousarray(np.stack(out))


def gen_mixed():
    """configs[2]'s per-GPU slice pinned on real mixed inputs: the
    reference's predict.py:58-91 flow on the 8 MIXED_IMAGES crops as ONE batch, the way
    config/daclip-sde/test.py:102-129 feeds DenoisingModel (encode_image(control=True) ->
    noise_state -> T=100 reverse_posterior -> tensor2img) with the restoration fixture's
    tracking UNet weights (w_g1 / w_g2 / k of restore_rain_256_t100.npz), seed-0 ViT-B/32
    DaCLIP, injected noise (restore_noise(tag="mx")), fp32 CPU; plus the degradation-class
    scores softmax(100 d^ t^T) over the 10 test.yml classes and their argmax
    (evaluate_daclip.py:45-50)."""
    from open_clip import tokenize
    from daclip_amd.preprocess import clip_transform
    rgb = mixed_crops()
    image = rgb / 255.0                                              # predict.py:64 (float64)
    img4clip = np.stack([clip_transform(im).numpy() for im in image])
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    ic, dc = d.encode_image(T(img4clip), control=True)
    ic, dc = ic.float(), dc.float()
    tf = d.encode_text(tokenize(DEGRADATIONS))
    dn = dc / dc.norm(dim=-1, keepdim=True)
    tn = tf / tf.norm(dim=-1, keepdim=True)
    probs = (100.0 * dn @ tn.T).softmax(dim=-1)
    lq = torch.tensor(image, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()   # predict.py:73-75
    g = np.load(os.path.join(HERE, "restore_rain_256_t100.npz"))
    m = ConditionalUNet(**unet_cfg(64)).eval()
    spec = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = synth.tracking_state_dict(synth.synth_state_dict(spec, 0), g["w_g1"], g["w_g2"], float(g["k"]))
    m.load_state_dict({k: T(v) for k, v in sd.items()}, strict=True)
    sde = ref_utils.IRSDE(max_sigma=50, T=MIXED_T, schedule="cosine", eps=0.005, device="cpu")
    sde.set_model(m)
    n0, steps = restore_noise(tuple(lq.shape), T=MIXED_T, tag="mx")
    with NoiseInjector([n0]):
        noisy = sde.noise_state(lq)
    sde.set_mu(lq)
    with NoiseInjector(list(steps)):
        out = sde.reverse_posterior(noisy, text_context=dc, image_context=ic).numpy()
    out_u8 = np.stack([ref_utils.tensor2img(T(o.copy())) for o in out])
    lq_u8 = np.stack([ref_utils.tensor2img(T(o.copy())) for o in lq.numpy()])
    psnr = np.array([ref_utils.calculate_psnr(a, b) for a, b in zip(out_u8, lq_u8)])
    inr = ((out > 0) & (out < 1)).mean(axis=(1, 2, 3))
    print(f"mixed: argmax {probs.argmax(-1).tolist()} psnr vs lq {np.round(psnr, 2).tolist()} "
          f"in-range {np.round(inr, 4).tolist()}", flush=True)
    np.savez_compressed(os.path.join(HERE, "mixed8_256_t100.npz"), names=np.array(MIXED_IMAGES),
                        classes=np.array(DEGRADATIONS), rgb_u8=rgb, img4clip=img4clip.astype(np.float32),
                        image_context=ic.numpy(), degra_context=dc.numpy(), probs=probs.numpy(),
                        argmax=probs.argmax(dim=-1).numpy(), out=out, out_u8=out_u8, lq_u8=lq_u8,
                        psnr_out_vs_lq=psnr)


def gen_variants():
    """Two sampler / context variants of the reference, 16x16 / 32x32:
    * sample_T != T: IRSDE(T=100, sample_T=50) -> 50-entry schedule and the model called at
      t * sample_scale = 2t (sde_utils.py:84-89, 297-313), posterior loop with injected noise;
    * image_context=None: every SpatialTransformer's attn2 becomes self-attention over
      norm2(x) (attention.py:174). That only runs when context_dim equals the channels of
      every SpatialTransformer level, so this UNet is nf=64, ch_mult [1,2,4,4], context 256."""
    m = ConditionalUNet(**unet_cfg(64)).eval()
    load(m, seed=0)
    sde = ref_utils.IRSDE(max_sigma=50, T=100, sample_T=50, schedule="cosine", eps=0.005, device="cpu")
    sde.set_model(m)
    b, h, w = 1, 16, 16
    lq = synth.synth_images(b, h, w, seed=81)
    tc = synth.synth_noise((b, 512), seed=3, tag="text") * 0.5
    ic = synth.synth_noise((b, 512), seed=4, tag="image") * 0.5
    x0 = lq + synth.synth_noise((b, 3, h, w), seed=82, tag="st_noisy") * (50 / 255)
    steps = synth.synth_noise((50, b, 3, h, w), seed=83, tag="st_steps")
    sde.set_mu(T(lq))
    with NoiseInjector(list(steps)):
        out = sde.reverse_posterior(T(x0), text_context=T(tc), image_context=T(ic)).numpy()
    out_s = {"st_lq": lq, "st_x0": x0, "st_tc": tc, "st_ic": ic, "st_steps": steps, "st_out": out,
             "st_thetas": sde.thetas.numpy(), "st_dt": np.float32(sde.dt.item())}

    cfg = dict(in_nc=3, out_nc=3, nf=64, ch_mult=[1, 2, 4, 4], context_dim=256,
               use_degra_context=True, use_image_context=True)
    m = ConditionalUNet(**cfg).eval()
    spec = load(m, seed=1)
    b, h, w = 2, 32, 32
    xt = synth.synth_noise((b, 3, h, w), seed=84, tag="sc_xt") * 0.3 + 0.5
    mu = synth.synth_images(b, h, w, seed=85)
    tc = synth.synth_noise((b, 256), seed=86, tag="sc_text") * 0.5
    out_s.update(sc_xt=xt, sc_mu=mu, sc_tc=tc,
                 sc_fwd=m(T(xt), T(mu), 31.0, text_context=T(tc), image_context=None).numpy(),
                 sc_fwd_notext=m(T(xt), T(mu), 7.0).numpy())
    sde = ref_utils.IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005, device="cpu")
    sde.set_model(m)
    sde.set_mu(T(mu))
    steps = synth.synth_noise((3, b, 3, h, w), seed=87, tag="sc_steps")
    with NoiseInjector(list(steps)):
        out_s["sc_loop3"] = sde.reverse_posterior(T(xt), T=3, text_context=T(tc)).numpy()
    out_s["sc_steps"] = steps
    np.savez_compressed(os.path.join(HERE, "sampler_variants.npz"), **out_s)
    json.dump({k: list(v) for k, v in spec.items()}, open(os.path.join(HERE, "selfctx_state_spec.json"), "w"))


def _daclip(vision, text, embed):
    d = DaCLIP(CLIP(embed_dim=embed, vision_cfg=vision, text_cfg=text)).eval()
    load(d, seed=0)
    return d


def gen_daclip():
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    img = synth.synth_noise((2, 3, 224, 224), seed=11, tag="img4clip")
    ic, dc = d.encode_image(T(img), control=True)
    np.savez_compressed(os.path.join(HERE, "daclip_b32_encode.npz"), img=img,
                        image_context=ic.numpy(), degra_context=dc.numpy())
    small_v = dict(image_size=64, layers=3, width=128, patch_size=32)
    small_t = dict(context_length=16, vocab_size=64, width=64, heads=2, layers=1)
    d = _daclip(small_v, small_t, 64)
    img = synth.synth_noise((3, 3, 64, 64), seed=12, tag="img4clip_small")
    ic, dc = d.encode_image(T(img), control=True)
    np.savez_compressed(os.path.join(HERE, "daclip_small_encode.npz"), img=img,
                        image_context=ic.numpy(), degra_context=dc.numpy())


def gen_plain_encode():
    """DaCLIP.encode_image(image) with the reference's default control=False
    (daclip_model.py:54-55 -> CLIP.encode_image, model.py:233-235): the clip tower alone."""
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    img = synth.synth_noise((2, 3, 224, 224), seed=11, tag="img4clip")
    out = dict(b32=d.encode_image(T(img)).numpy(), b32_norm=d.encode_image(T(img), normalize=True).numpy())
    small_v = dict(image_size=64, layers=3, width=128, patch_size=32)
    small_t = dict(context_length=16, vocab_size=64, width=64, heads=2, layers=1)
    d = _daclip(small_v, small_t, 64)
    img = synth.synth_noise((3, 3, 64, 64), seed=12, tag="img4clip_small")
    out["small"] = d.encode_image(T(img)).numpy()
    np.savez_compressed(os.path.join(HERE, "daclip_plain_encode.npz"), **out)


DEGRADATIONS = ["motion-blurry", "hazy", "jpeg-compressed", "low-light", "noisy", "raindrop",
                "rainy", "shadowed", "snowy", "uncompleted"]   # options/test.yml:4 order


def text_images():
    """The 6 encoder inputs of text_b32.npz (regenerated by the tests, not stored)."""
    img = synth.synth_noise((6, 3, 224, 224), seed=31, tag="img4clip_text")
    img[3:] = np.clip(img[3:] * 0.2 + synth.synth_images(3, 224, 224, seed=32), -3, 3)
    return img


def gen_text():
    """Text tower + degradation-class scoring (daclip_model.py:125-126 -> model.py:237-249;
    evaluate_daclip.py:45-50, 78-84): token ids from the reference tokenizer for the 10
    class names, encode_text features, and softmax(100 d^ t^T) / argmax for 6 images."""
    from open_clip import tokenize
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-B-32.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    tokens = tokenize(DEGRADATIONS)
    tf = d.encode_text(tokens)
    img = text_images()
    _, dc = d.encode_image(T(img), control=True)
    dn = dc / dc.norm(dim=-1, keepdim=True)
    tn = tf / tf.norm(dim=-1, keepdim=True)
    probs = (100.0 * dn @ tn.T).softmax(dim=-1)
    extra = ["A photo of heavy rain!", "it's a JPEG-compressed image, isn't it?", "3x3 conv &amp; 512px",
             "café  crème\tbrûlée", "low light " * 40]
    np.savez_compressed(os.path.join(HERE, "text_b32.npz"), classes=np.array(DEGRADATIONS),
                        extra_texts=np.array(extra), extra_tokens=tokenize(extra).numpy(),
                        tokens=tokens.numpy(), text_features=tf.numpy(), degra=dc.numpy(),
                        probs=probs.numpy(), argmax=probs.argmax(dim=-1).numpy())
    small_v = dict(image_size=64, layers=3, width=128, patch_size=32)
    small_t = dict(context_length=16, vocab_size=64, width=64, heads=2, layers=1)
    d = _daclip(small_v, small_t, 64)
    rng = np.random.default_rng(5)
    tok = rng.integers(1, 62, size=(4, 16)).astype(np.int64)
    for i, e in enumerate([3, 9, 15, 6]):                 # EOT (highest id) at varied positions
        tok[i, e] = 63
        tok[i, e + 1:] = 0
    tf = d.encode_text(T(tok))
    np.savez_compressed(os.path.join(HERE, "text_small.npz"), tokens=tok, text_features=tf.numpy())


def wild_images():
    """Encoder input of wild_l14_encode.npz (regenerated by the tests, not stored)."""
    return synth.synth_noise((1, 3, 224, 224), seed=41, tag="img4clip_wild")


def gen_wild():
    """Wild-IR (BASELINE config 4 model): ConditionalUNet(scale=0.5, context 768, image context
    only; config/wild-ir/options/inference.yml:30-39) forwards and the ViT-L/14 DaCLIP
    encode_image(control=True) (wild-daclip_ViT-L-14, inference.py:68-96)."""
    WildUNet = _refimport.import_wild_unet()
    setting = dict(in_nc=3, out_nc=3, nf=64, ch_mult=[1, 2, 4, 8], context_dim=768,
                   use_degra_context=False, use_image_context=True, scale=0.5)
    m = WildUNet(**setting).eval()
    spec = load(m, seed=0)
    json.dump({k: list(v) for k, v in spec.items()}, open(os.path.join(HERE, "wild_state_spec.json"), "w"))
    out = {}
    for tag, (B, H, W) in (("32x32", (1, 32, 32)), ("48x40", (2, 48, 40))):
        xt = synth.synth_noise((B, 3, H, W), seed=51, tag="wx" + tag) * 0.3 + 0.5
        mu = synth.synth_images(B, H, W, seed=52)
        ic = synth.synth_noise((B, 768), seed=53, tag="wic" + tag)
        out[f"{tag}_xt"], out[f"{tag}_mu"], out[f"{tag}_ic"] = xt, mu, ic
        out[f"{tag}_out"] = m(T(xt), T(mu), 37.0, image_context=T(ic)).numpy()
    np.savez_compressed(os.path.join(HERE, "wild_unet_fwd.npz"), **out)
    cfg = json.load(open(_refimport.REF + "/open_clip/model_configs/daclip_ViT-L-14.json"))
    d = _daclip(cfg["vision_cfg"], cfg["text_cfg"], cfg["embed_dim"])
    ic, dc = d.encode_image(T(wild_images()), control=True)
    np.savez_compressed(os.path.join(HERE, "wild_l14_encode.npz"), image_context=ic.numpy(),
                        degra_context=dc.numpy())


def gen_modules():
    """Per-module fixtures (small shapes) used to localise kernel bugs."""
    from models.modules.module_util import ResBlock, LinearAttention, default_conv, NonLinearity
    from models.modules.attention import SpatialTransformer
    import functools
    out = {}
    rb = functools.partial(ResBlock, conv=default_conv, act=NonLinearity())
    for tag, din, dout in (("rb64", 64, 64), ("rb96_32", 96, 32)):
        m = rb(dim_in=din, dim_out=dout, time_emb_dim=256).eval()
        load(m, seed=5)
        x = synth.synth_noise((2, din, 12, 10), seed=13, tag=tag)
        te = synth.synth_noise((2, 256), seed=14, tag=tag + "t")
        out[f"{tag}_x"], out[f"{tag}_t"] = x, te
        out[f"{tag}_y"] = m(T(x), T(te)).numpy()
    la = LinearAttention(64).eval()
    load(la, seed=5)
    x = synth.synth_noise((2, 64, 16, 12), seed=15, tag="la")
    out["la_x"], out["la_y"] = x, la(T(x)).numpy()
    st = SpatialTransformer(64, 2, 32, depth=1, context_dim=512).eval()
    load(st, seed=5)
    x = synth.synth_noise((2, 64, 8, 8), seed=16, tag="st")
    c = synth.synth_noise((2, 1, 512), seed=17, tag="stc")
    out["st_x"], out["st_c"], out["st_y"] = x, c, st(T(x), context=T(c)).numpy()
    np.savez_compressed(os.path.join(HERE, "modules.npz"), **out)


def gen_img_metrics():
    a = synth.synth_images(1, 24, 20, seed=21)[0]
    b = np.clip(a + 0.03 * synth.synth_noise(a.shape, seed=22, tag="pert"), -0.1, 1.1)
    ua = ref_utils.tensor2img(T(a.copy()))
    ub = ref_utils.tensor2img(T(b.copy()))
    from data.util import bgr2ycbcr          # data/util.py:189-210 (no cv2 call on this path)
    fa = ua.astype(np.float64) / 255.0
    np.savez_compressed(os.path.join(HERE, "img_metrics.npz"), a=a, b=b, ua=ua, ub=ub,
                        psnr=np.float64(ref_utils.calculate_psnr(ua, ub)),
                        y_u8=bgr2ycbcr(ua.copy(), only_y=True), ycc_u8=bgr2ycbcr(ua.copy(), only_y=False),
                        y_f=bgr2ycbcr(fa.copy(), only_y=True), ycc_f=bgr2ycbcr(fa.copy(), only_y=False))


if __name__ == "__main__":
    which = sys.argv[1:] or ["spec", "unet", "sde", "daclip", "text", "wild", "modules", "img"]
    fns = dict(spec=gen_state_spec, unet=gen_unet_forward, sde=gen_sde, daclip=gen_daclip,
               text=gen_text, wild=gen_wild, modules=gen_modules, img=gen_img_metrics,
               headline=gen_headline, variants=gen_variants, restore=gen_restore,
               plain=gen_plain_encode, mixed=gen_mixed)
    for w in which:
        print("generating", w, flush=True)
        fns[w]()
