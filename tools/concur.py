"""Does running the batch as two concurrent half-batch graph loops on two streams beat one loop?

tools/concur.py [--T 100] [--iters 3]: times (a) one B=8 posterior loop, (b) two B=4 loops on one
stream, (c) two B=4 loops on two streams at once (separate UNet handles, same weights).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "da-clip_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--T", type=int, default=100)
    p.add_argument("--iters", type=int, default=3)
    a = p.parse_args()
    from daclip_amd import arch, synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    dev = torch.device("cuda", 0)
    spec = arch.unet_state_spec(arch.UNetConfig())
    sd = {k: torch.from_numpy(v).to(dev) for k, v in synth.synth_state_dict(spec, 0).items()}
    kw = dict(context_dim=512, use_degra_context=True, use_image_context=True)

    def make(B):
        u = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], **kw, device=dev, dtype="bf16")
        u.load_state_dict(sd)
        s = IRSDE(max_sigma=50, T=a.T, schedule="cosine", eps=0.005)
        s.set_model(u)
        lq = torch.from_numpy(synth.synth_images(B, 256, 256, seed=100)).to(dev)
        s.set_mu(lq)
        g = torch.Generator().manual_seed(5)
        ic = torch.randn(B, 512, generator=g).to(dev)
        dc = torch.randn(B, 512, generator=g).to(dev)
        x = s.noise_state(lq)
        return s, x, ic, dc

    full = make(8)
    halves = [make(4), make(4)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(s, x, ic, dc):
        return s.reverse_posterior(x, text_context=dc, image_context=ic)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.iters * 1e3

    def two_streams():
        cur = torch.cuda.current_stream(dev)
        for st, h in zip(streams, halves):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                run(*h)
        for st in streams:
            cur.wait_stream(st)

    print(f"B=8 one loop          {timed(lambda: run(*full)):8.1f} ms", flush=True)
    print(f"2 x B=4, one stream   {timed(lambda: [run(*h) for h in halves]):8.1f} ms", flush=True)
    print(f"2 x B=4, two streams  {timed(two_streams):8.1f} ms", flush=True)


if __name__ == "__main__":
    main()
