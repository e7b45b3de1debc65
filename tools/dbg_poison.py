import os, sys
os.environ["DAC_POISON"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import numpy as np, torch
from daclip_amd.unet import ConditionalUNet
from daclip_amd.sde import IRSDE
from daclip_amd.open_clip import DaCLIP
from daclip_amd import arch
g = np.load(os.path.join(ROOT, "tests/golden/posterior_loop_16x16.npz"))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
for dt in ("fp32", "bf16"):
    m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=dt); m.load_synthetic(0)
    for (B, S) in ((1, 16), (2, 32), (1, 30), (2, 256)):
        torch.manual_seed(0)
        x = torch.rand(B, 3, S, S, device="cuda"); mu = torch.rand(B, 3, S, S, device="cuda")
        tc = torch.randn(B, 512, device="cuda"); ic = torch.randn(B, 512, device="cuda")
        e = m(x, mu, 9.0, text_context=tc, image_context=ic)
        sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_mu(mu); sde.set_model(m)
        o = sde.reverse_posterior(x, T=3, text_context=tc, image_context=ic)
        print(dt, B, S, "forward finite", bool(torch.isfinite(e).all()), "loop finite", bool(torch.isfinite(o).all()), flush=True)
    c = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, dtype=dt); c.load_synthetic(0)
    i1, d1 = c.encode_image(torch.randn(2, 3, 224, 224, device="cuda"), control=True)
    print(dt, "encode finite", bool(torch.isfinite(i1).all() and torch.isfinite(d1).all()), flush=True)
