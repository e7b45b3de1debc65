"""Multi-process (gloo, CPU) tests of the data-parallel sharding layer (daclip_amd/shard.py).

The per-image restore used here is the oracle's posterior loop with a stand-in noise
predictor and noise keyed by GLOBAL image index, the same contract the HIP path keeps via
dac_set_noise_offset; the property checked is that sharded + gathered == unsharded, bit-exact,
for even and uneven splits, plus the weight broadcast."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from daclip_amd import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds_cover_and_balance():
    for n in range(0, 40):
        for w in range(1, 9):
            b = [shard.shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            sz = [hi - lo for lo, hi in b]
            assert max(sz) - min(sz) <= 1 and sz == sorted(sz, reverse=True)
    with pytest.raises(ValueError):
        shard.shard_bounds(4, 2, 2)


def _restore_oracle(lq, first, T=4):
    """Oracle posterior loop; eps from a fixed per-pixel function of (x, mu), noise keyed by
    global image index (so the result of image g never depends on the shard layout)."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import sde as OS
    from daclip_amd import synth
    s = OS.IRSDE(50, T, "cosine", 0.005)
    out = []
    for j in range(lq.shape[0]):
        g = first + j
        mu = lq[j:j + 1].numpy()
        s.mu = mu
        x = s.noise_state(mu, synth.synth_noise(mu.shape, seed=1000 + g, tag="ns"))
        for i, t in enumerate(range(T, 0, -1)):
            eps = np.tanh(3.0 * (x - mu)).astype(np.float32)
            x = s.posterior_step(x, eps, t, synth.synth_noise(mu.shape, seed=2000 + g, tag=f"z{i}"))
        out.append(torch.from_numpy(np.ascontiguousarray(x, np.float32)))
    return torch.cat(out, 0) if out else lq[:0].clone()


def _worker(rank, ws, port, n_img, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from daclip_amd import arch, synth
        spec = arch.unet_state_spec(arch.UNetConfig(nf=16, ch_mult=(1, 2)))
        keys = list(spec)
        sd = synth.synth_state_dict(spec, 7) if rank == 0 else None
        got = shard.broadcast_state(sd, keys, "cpu")
        ref = synth.synth_state_dict(spec, 7)
        bc_ok = all(np.array_equal(got[k].numpy(), np.asarray(ref[k], np.float32)) for k in keys)
        lq = torch.from_numpy(synth.synth_images(n_img, 8, 8, seed=5))
        out = shard.restore_sharded(_restore_oracle, lq)
        q.put((rank, bc_ok, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,n_img", [(2, 4), (2, 5), (3, 2)])
def test_gloo_sharded_restore_equals_unsharded(ws, n_img):
    from daclip_amd import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, n_img, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lq = torch.from_numpy(synth.synth_images(n_img, 8, 8, seed=5))
    ref = _restore_oracle(lq, 0).numpy()
    for rank, bc_ok, out in res:
        assert bc_ok, f"rank {rank}: broadcast weights differ"
        assert out.shape == ref.shape
        assert np.array_equal(out, ref), f"rank {rank}: sharded restore differs"
