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
sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_mu(mu)
def run():
    xx = x.clone(); es = []; xs = []
    for i, t in enumerate(range(5, 0, -1)):
        e = m(xx, mu, float(t), **kw); es.append(e.clone())
        xx = sde.step(0, xx, e, mu, z[i], t); xs.append(xx.clone())
    return es, xs
runs = [run() for _ in range(4)]
for k in range(1, 4):
    print("run", k, "eps diffs", [float((runs[k][0][i] - runs[0][0][i]).abs().max()) for i in range(5)],
          "x diffs", [float((runs[k][1][i] - runs[0][1][i]).abs().max()) for i in range(5)], flush=True)
# determinism of step alone
e0 = runs[0][0][0]
s1 = [sde.step(0, x, e0, mu, z[0], 5) for _ in range(5)]
print("step repeat", [float((s - s1[0]).abs().max()) for s in s1], flush=True)
# forward alone on runs[0] x states
for i, t in enumerate(range(4, 0, -1)):
    xi = runs[0][1][i]
    es = [m(xi, mu, float(t), **kw) for _ in range(4)]
    print("fwd repeat t", t, [float((e - es[0]).abs().max()) for e in es], "vs run0", float((es[0] - runs[0][0][i + 1]).abs().max()), flush=True)
