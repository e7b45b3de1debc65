"""One fp16 UNet forward at batch B (argv[1]) -- run under rocprofv3 to list the kernels a batch
size selects (tools/inv_probe.py finds the batch sizes whose outputs differ)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
import torch  # noqa: E402
from daclip_amd import arch, synth  # noqa: E402
from daclip_amd.unet import ConditionalUNet  # noqa: E402

B = int(sys.argv[1])
sd = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
m = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, dtype="fp16")
m.load_state_dict(sd)
x = T(synth.synth_noise((B, 3, 256, 256), seed=101, tag="b16") * 0.3 + 0.5)
mu = T(synth.synth_images(B, 256, 256, seed=102))
tc = T(synth.synth_noise((B, 512), seed=103, tag="tc"))
ic = T(synth.synth_noise((B, 512), seed=104, tag="ic"))
out = m(x, mu, 42.0, text_context=tc, image_context=ic)
torch.cuda.synchronize()
print("ok", out.shape)
