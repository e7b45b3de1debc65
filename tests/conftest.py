import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "da-clip_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name))
    return load


@pytest.fixture(scope="session")
def unet_sd():
    from daclip_amd import arch, synth
    return synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)


@pytest.fixture(scope="session")
def restore_fixture():
    """tests/golden/restore_rain_256_t100.npz (make_golden.py gen_restore) with its UNet weights
    (synth.tracking_state_dict over the seed-0 synthetic weights) and injected noises."""
    import numpy as np
    from daclip_amd import arch, synth
    g = dict(np.load(os.path.join(GOLDEN, "restore_rain_256_t100.npz")))
    base = synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), seed=0)
    sd = synth.tracking_state_dict(base, g["w_g1"], g["w_g2"], float(g["k"]))
    shape = (1, 3, 256, 256)
    noise = dict(n0=synth.synth_noise(shape, seed=91, tag="rs_noise_state"),
                 steps=synth.synth_noise((100,) + shape, seed=92, tag="rs_steps"),
                 n0_64=synth.synth_noise((1, 3, 64, 64), seed=91, tag="sde64_noise_state"),
                 steps_64=synth.synth_noise((100, 1, 3, 64, 64), seed=92, tag="sde64_steps"))
    return g, sd, noise
