import os, sys, ctypes, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch
from daclip_amd import arch, synth, _lib
from daclip_amd.unet import ConditionalUNet
from daclip_amd.sde import IRSDE
m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype="bf16")
m.load_synthetic(0)
sde = IRSDE(50, 100, schedule="cosine", eps=0.005); sde.set_model(m)
B, R = 2, 64
lq = torch.rand(B, 3, R, R, device="cuda"); sde.set_mu(lq)
tc = torch.randn(B, 512, device="cuda"); ic = torch.randn(B, 512, device="cuda")
x = sde.reverse_posterior(lq, T=3, text_context=tc, image_context=ic); torch.cuda.synchronize()
print("no-prof ok", x.abs().mean().item(), flush=True)
h = m._h
print("enable", _lib.lib().dac_profile_enable(h.h, int(sys.argv[1]) if len(sys.argv) > 1 else 301), flush=True)
x = sde.reverse_posterior(lq, T=3, text_context=tc, image_context=ic)
print("after launch err:", _lib.lib().dac_last_error(h.h), flush=True)
torch.cuda.synchronize()
print("synced", flush=True)
a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
n = _lib.lib().dac_profile_read(h.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
print("read", n, a.value, b.value, c.value, _lib.lib().dac_last_error(h.h), flush=True)
