import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import numpy as np, torch
from daclip_amd.unet import ConditionalUNet
g = np.load(os.path.join(ROOT, "tests/golden/posterior_loop_16x16.npz"))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
for dt in ("fp32", "bf16"):
  for size in (16, 64):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt); m.load_synthetic(0)
    kw = dict(text_context=T(g["text_context"]), image_context=T(g["image_context"]))
    torch.manual_seed(0)
    x = torch.rand(1, 3, size, size, device="cuda"); mu = torch.rand(1, 3, size, size, device="cuda")
    ref = m(x, mu, 7.0, **kw)
    bad = 0
    for k in range(30):
        # perturb arena contents with a different input / time
        m(torch.randn_like(x) * (k + 1), mu, float(k + 1), **kw)
        o = m(x, mu, 7.0, **kw)
        d = float((o - ref).abs().max())
        if d != 0: bad += 1
        if d != 0 and bad < 4: print(dt, size, "iter", k, "diff", d, flush=True)
    print(dt, size, "nondeterministic runs:", bad, "/ 30", flush=True)
