"""CPU oracle for the DA-CLIP + IR-SDE hot path — TEST INFRASTRUCTURE ONLY.

A numpy fp32 restatement of the reference algorithm (each function cites the reference
file:line it follows). It is pinned against golden fixtures produced by running the
reference itself in the build container (tests/golden/make_golden.py; fixtures under
tests/golden/*.npz; tests/test_oracle.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / CPU baseline. The product path (da-clip_amd/) never
imports it and has no CPU fallback.
"""
from . import clip, imgs, nn, sde, unet  # noqa: F401
