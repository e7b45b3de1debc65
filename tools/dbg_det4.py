import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import numpy as np, torch
from daclip_amd.unet import ConditionalUNet
from daclip_amd.sde import IRSDE
g = np.load(os.path.join(ROOT, "tests/golden/posterior_loop_16x16.npz"))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype="fp32"); m.load_synthetic(0)
kw = dict(text_context=T(g["text_context"]), image_context=T(g["image_context"]))
x = T(g["noisy"]); mu = T(g["lq"]); z = T(g["step_noise"][:5])
sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_mu(mu); sde.set_model(m)
e1 = m(x, mu, 2.0, **kw)
a3 = sde.reverse_posterior(x, T=3, noises=z[:3], **kw)
e2 = m(x, mu, 2.0, **kw)
print("eager before/after graph", float((e1 - e2).abs().max()), flush=True)
b3 = sde.reverse_posterior(x, T=3, noises=z[:3], **kw)
print("graph T=3 repeat", float((a3 - b3).abs().max()), flush=True)
torch.cuda.synchronize()
c3 = sde.reverse_posterior(x, T=3, noises=z[:3], **kw); torch.cuda.synchronize()
print("graph T=3 repeat synced", float((a3 - c3).abs().max()), flush=True)
# graph vs eager-manual per step for T=3 using T=1,2,3 graphs
xx = x.clone()
for i, t in enumerate(range(3, 0, -1)):
    e = m(xx, mu, float(t), **kw)
    xx = sde.step(0, xx, e, mu, z[i], t)
print("graph T=3 vs manual", float((a3 - xx).abs().max()), float((c3 - xx).abs().max()), flush=True)
