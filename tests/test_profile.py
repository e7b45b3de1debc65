"""The bench's roofline measurement (bench.py dominant_roofline / graph_profile, engine.cpp
profile_graph, common.h StampGuard): every conv launch of one restore timed INSIDE a replay of the
captured loop graph by wall-clock stamps the kernels write themselves.

CPU: the time-sharing attribution over overlapping launches. GPU: the stamped replay has exactly
the timed graph's launches (same count per step for every symbol, branch launches flagged), every
launch's duration and symbol are filled in, the stamps do not perturb the replay, and the result
of the profiled restore equals an unprofiled one bit for bit."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def _row(ms, t0, fl=1.0, cls=312, sym="k", br=0):
    # (ms, flops, bytes, class, label, symbol, start ms, in-branch) as bench._launch_rows returns
    return (ms, fl, 0.0, cls, "", sym, t0, br)


def test_time_shares_divides_overlap():
    import bench
    rows = [_row(2.0, 0.0), _row(2.0, 1.0), _row(1.0, 5.0)]
    sh = bench.time_shares(rows)
    # [0,1) alone, [1,2) shared by two, [2,3) alone; the third launch alone
    assert sh == pytest.approx([1.5, 1.5, 1.0])
    assert sum(sh) == pytest.approx(4.0)           # = busy time of the union
    g = bench._group(rows, lambda c, s: s, sh)
    assert g["k"]["launches"] == 3 and g["k"]["ms"] == pytest.approx(5.0) and g["k"]["share_ms"] == pytest.approx(4.0)


def test_time_shares_nested_and_identical_intervals():
    import bench
    rows = [_row(4.0, 0.0), _row(1.0, 1.0), _row(4.0, 0.0)]
    sh = bench.time_shares(rows)
    # [0,1): 2 active, [1,2): 3 active, [2,4): 2 active
    assert sh == pytest.approx([0.5 + 1 / 3 + 1.0, 1 / 3, 0.5 + 1 / 3 + 1.0])
    assert sum(sh) == pytest.approx(4.0)


@pytest.mark.gpu
def test_graph_profile_matches_timed_graph():
    import bench
    from daclip_amd import arch, synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.sde import IRSDE
    dev = torch.device("cuda", 0)
    T, B, R = 4, 4, 64
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, device=dev, dtype="fp16")
    unet.load_state_dict(synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), 0))
    clip = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, device=dev, dtype="fp16", with_text=False)
    clip.load_synthetic(seed=0)
    sde = IRSDE(max_sigma=50, T=T, schedule="cosine", eps=0.005)
    sde.set_model(unet)
    n, lo, lq, img = bench.shard_inputs(B, R, 1, 0, dev)
    n0 = torch.from_numpy(synth.synth_noise((B, 3, R, R), seed=5, tag="tp_n0")).to(dev)
    zs = torch.from_numpy(synth.synth_noise((T, B, 3, R, R), seed=6, tag="tp_z")).to(dev)
    sde.set_mu(lq)
    ic, dc = clip.encode_image(img, control=True)

    def step():                                     # injected noise: a deterministic restore
        return sde.reverse_posterior(sde.noise_state(lq, noise=n0), noises=zs, text_context=dc, image_context=ic)
    ref = step().clone()
    torch.cuda.synchronize()
    rows, graph_ms, step_ms = bench.graph_profile(unet._h, step)
    out = step()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)                    # profiling left the handle's graph untouched
    assert rows and len(rows) % T == 0
    per = len(rows) // T
    for k in range(T):                              # every step records the same launches
        assert [r[5] for r in rows[k * per:(k + 1) * per]] == [r[5] for r in rows[:per]]
    assert all(r[0] > 0 and r[1] > 0 and r[5] for r in rows), "duration / flops / symbol missing"
    assert any(r[7] for r in rows) and not all(r[7] for r in rows)   # split section flagged
    assert all(r[6] >= 0 for r in rows) and graph_ms > 0
    assert sum(r[0] for r in rows[:per]) < graph_ms / T * 2.5        # durations are per launch
    # the stamped profile of the same handle again: same launches, same symbols
    rows2, _, _ = bench.graph_profile(unet._h, step)
    assert [r[5] for r in rows2] == [r[5] for r in rows]
    r = bench.dominant_roofline(unet._h, step, "fp16", step_ms)
    assert r["kernel"] and 0 < r["frac"] <= r["frac_time_shared"] < 1.0 and r["launches_per_restore"] > 0
