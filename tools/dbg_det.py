import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import numpy as np, torch
from daclip_amd import arch, synth
from daclip_amd.unet import ConditionalUNet
from daclip_amd.sde import IRSDE
g = np.load(os.path.join(ROOT, "tests/golden/posterior_loop_16x16.npz"))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
for dt in ("fp32", "bf16"):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt); m.load_synthetic(0)
    kw = dict(text_context=T(g["text_context"]), image_context=T(g["image_context"]))
    x = T(g["noisy"]); mu = T(g["lq"])
    outs = [m(x, mu, 5.0, **kw) for _ in range(4)]
    print(dt, "eager repeat max diff", [float((o - outs[0]).abs().max()) for o in outs], flush=True)
    sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_mu(mu)
    z = T(g["step_noise"][:1])
    sde.set_model(m); a = sde.reverse_posterior(x, T=1, noises=z, **kw)
    sde.set_model(lambda *q, **k: m(*q, **k)); b = sde.reverse_posterior(x, T=1, noises=z, **kw)
    print(dt, "T=1 graph vs python", float((a - b).abs().max()), flush=True)
    sde.set_model(m); a2 = sde.reverse_posterior(x, T=1, noises=z, **kw)
    print(dt, "graph repeat", float((a - a2).abs().max()), flush=True)
    # eps from graph path: x1 = posterior(x, eps); recover eps and compare to eager
print("---- multi-step", flush=True)
for dt in ("fp32",):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt); m.load_synthetic(0)
    kw = dict(text_context=T(g["text_context"]), image_context=T(g["image_context"]))
    x = T(g["noisy"]); mu = T(g["lq"])
    for nT in (2, 3, 5):
        sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_mu(mu)
        z = T(g["step_noise"][:nT])
        sde.set_model(m); a = sde.reverse_posterior(x, T=nT, noises=z, **kw)
        sde.set_model(lambda *q, **k: m(*q, **k)); b = sde.reverse_posterior(x, T=nT, noises=z, **kw)
        # manual loop with eager forward + python math
        xx = x.clone()
        for i, t in enumerate(range(nT, 0, -1)):
            e = m(xx, mu, float(t), **kw)
            xx = sde.step(0, xx, e, mu, z[i], t)
        print(nT, "graph-py", float((a - b).abs().max()), "graph-manual", float((a - xx).abs().max()), "py-manual", float((b - xx).abs().max()), flush=True)
