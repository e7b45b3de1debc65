"""Per-shape timing of every conv launch in one restore of the bench batch (eager replay with
HIP events around each launch; report printed by the library to stderr).
Usage: python tools/conv_profile.py [--dtype bf16] [--batch 8] [--res 256] [--T 2]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch  # noqa: E402
from daclip_amd import arch, synth, _lib  # noqa: E402
from daclip_amd.unet import ConditionalUNet  # noqa: E402
from daclip_amd.sde import IRSDE  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--res", type=int, default=256)
ap.add_argument("--T", type=int, default=2)
a = ap.parse_args()
m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype=a.dtype)
m.load_synthetic(0)
B, R = a.batch, a.res
lq = torch.from_numpy(synth.synth_images(B, R, R, seed=1)).cuda()
c = torch.from_numpy(synth.synth_noise((B, 512), seed=2, tag="c")).cuda()
s = IRSDE(50, 100, schedule="cosine", eps=0.005)
s.set_model(m)
s.set_mu(lq)
s.reverse_posterior(lq, T=a.T, text_context=c, image_context=c)   # capture + warm
h = m._h
h.check(_lib.lib().dac_profile_enable(h.h, 999), "profile_enable")
s.reverse_posterior(lq, T=a.T, text_context=c, image_context=c)
ms, fl, by = _lib.ctypes.c_double(), _lib.ctypes.c_double(), _lib.ctypes.c_double()
h.check(_lib.lib().dac_profile_read(h.h, _lib.ctypes.byref(ms), _lib.ctypes.byref(fl), _lib.ctypes.byref(by)), "read")
torch.cuda.synchronize()
