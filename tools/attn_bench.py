"""Standalone timing of the SpatialTransformer attention core (dac_op_attention) at the UNet's
32x32-level shapes: python tools/attn_bench.py [iters] [batch] [variants]. Prints us per call and
TFLOP/s (batch 8 by default; the split section runs 4 per branch; variants comma-separated)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch  # noqa: E402
from daclip_amd import _lib  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 50
BATCH = int(sys.argv[2]) if len(sys.argv) > 2 else 8
VARIANTS = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 3, 8, 11, 12]
L_ = _lib.lib()
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for (B, L, H), (tdt, code) in [(s, d) for s in [(BATCH, 1024, 16), (BATCH, 1024, 8)]
                               for d in [(torch.float16, _lib.DAC_F16), (torch.bfloat16, _lib.DAC_BF16)]]:
    qkv = torch.randn(B * L, 3 * H * 32, device="cuda").to(tdt)
    out = torch.empty(B * L, H * 32, device="cuda", dtype=tdt)
    pre = qkv.float()
    pre.view(B * L, 3, H * 32)[:, 0] *= 32 ** -0.5 * 1.4426950408889634
    pre = pre.to(tdt)
    for variant in VARIANTS:          # 8 | v: q prescaled (the engine's form)
        q = pre if variant & 8 else qkv
        args = (ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(out.data_ptr()), B, L, H, code, variant, st)
        for _ in range(3):
            L_.dac_op_attention(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            L_.dac_op_attention(*args)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / it
        fl = 4.0 * B * H * L * L * 32
        print(f"{str(tdt)[6:]} B={B} L={L} H={H} variant={variant}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
