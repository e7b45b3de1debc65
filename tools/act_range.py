"""Dynamic range of every stored UNet activation, fp32 (numpy oracle; CPU), for the fp16-mode
headroom note in DESIGN.md (fp16 saturates at 65504).

Instruments the oracle's ops (conv2d / linear / norms / softmax / SiLU / GELU / concatenation
results) and records, per op role, the largest |value| any call produced, over UNet forwards
at several timesteps of two workloads:
  rain:  the restoration fixture (tests/golden/restore_rain_256_t100.npz; tracking weights,
         the reference's contexts), x_t from noise_state at t=100 and the reference's x_{t=1};
  bench: the bench's seeded random-init weights on a synthetic LQ (the diverging headline case),
         x_t from noise_state at t=100 and 50.
    python tools/act_range.py [--res 256] > profiles/r04_act_range.txt
"""
import argparse
import os
import sys
import traceback
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]

import numpy as np  # noqa: E402

from oracle import nn as F, unet as OU, sde as OS  # noqa: E402
from daclip_amd import arch, synth  # noqa: E402

MAXABS = defaultdict(float)


def role():
    """The innermost oracle/unet.py function on the stack (resblock, linear_attention, ...)."""
    for fr in reversed(traceback.extract_stack()[:-2]):
        if fr.filename.endswith(os.path.join("oracle", "unet.py")):
            return fr.name
    return "?"


def wrap(name):
    f = getattr(F, name)

    def g(*a, **k):
        y = f(*a, **k)
        # 4-D results are NCHW activations (stored in the handle's dtype); 2-/3-D ones are the
        # fp32 per-step tables (time / prompt MLPs) or [B, L, C] token activations.
        key = f"{role()}:{name}:{np.ndim(y)}d"
        MAXABS[key] = max(MAXABS[key], float(np.abs(y).max()))
        return y
    setattr(F, name, g)


for n in ("conv2d", "linear", "silu", "gelu", "softmax", "layer_norm", "channel_layer_norm", "group_norm",
          "upsample_nearest2x"):
    wrap(n)


def run(tag, sd, lq, ic, dc, xts):
    for t, xt in xts:
        before = dict(MAXABS)
        out = OU.forward(sd, xt, lq, float(t), dc, ic)
        print(f"# {tag} t={t}: |x_t| max {np.abs(xt).max():.3g}, |eps| max {np.abs(out).max():.3g}", flush=True)
        del before


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=256)
    a = ap.parse_args()
    spec = arch.unet_state_spec(arch.UNetConfig())
    g = np.load(os.path.join(ROOT, "tests", "golden", "restore_rain_256_t100.npz"))
    sd = synth.tracking_state_dict(synth.synth_state_dict(spec, 0), g["w_g1"], g["w_g2"], float(g["k"]))
    lq = (g["rgb_u8"] / 255.0).astype(np.float32).transpose(2, 0, 1)[None]
    s = OS.IRSDE(50, 100, "cosine", 0.005)
    s.mu = lq
    x100 = s.noise_state(lq, synth.synth_noise(lq.shape, seed=91, tag="rs_noise_state"))
    run("rain", sd, lq, g["image_context"], g["degra_context"], [(100, x100), (1, g["x_t1"])])
    rain = dict(MAXABS)
    MAXABS.clear()
    sd0 = synth.synth_state_dict(spec, 0)
    lqb = synth.synth_images(1, a.res, a.res, seed=100)
    s.mu = lqb
    xb = s.noise_state(lqb, synth.synth_noise(lqb.shape, seed=5, tag="ar"))
    ctx = synth.synth_noise((1, 512), seed=6, tag="ar_ctx")
    run("bench", sd0, lqb, ctx, ctx, [(100, xb), (50, xb * 0.5 + lqb * 0.5)])
    print("# 4d = NCHW activations, 3d = [B,L,C] SpatialTransformer tokens (both stored in T);")
    print("# 2d = fp32 per-step tables (time / prompt MLPs, ResBlock scale-shift rows), never stored in T")
    print(f"{'op role':42s} {'rain max|v|':>12s} {'bench max|v|':>12s} {'headroom to 65504':>18s}")
    for k in sorted(set(rain) | set(MAXABS)):
        m = max(rain.get(k, 0.0), MAXABS.get(k, 0.0))
        print(f"{k:42s} {rain.get(k, 0.0):12.4g} {MAXABS.get(k, 0.0):12.4g} {65504.0 / max(m, 1e-30):17.1f}x")


if __name__ == "__main__":
    main()
