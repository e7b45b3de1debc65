"""bench.py's own multi-rank wiring on gloo (CPU, world size 2 and 3): shard_inputs ->
make_step (encode -> noise_state -> posterior loop -> all-gather) -> timed_steps (barriers,
max-over-ranks time). The restore is a stand-in with the HIP path's contract: contexts per
image, noise keyed by GLOBAL image index through sde.image_offset (dac_set_noise_offset on
the GPU), so the gathered batch must equal the single-rank batch bit for bit and every rank
must report the same (max) time. What stays unmeasured on hardware is the RCCL leg itself
(DESIGN.md §7)."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Clip:
    """encode_image(control=True) stand-in: per-image contexts from the image itself."""
    def encode_image(self, img, control=True):
        assert control
        m = img.mean(dim=(1, 2, 3))
        return m[:, None].repeat(1, 8), (-m)[:, None].repeat(1, 8)


class _SDE:
    """IRSDE stand-in: the oracle's schedule and posterior step, eps a fixed function of
    (x, mu, contexts), every draw keyed by global image index = image_offset + j."""
    T = 3

    def __init__(self):
        sys.path.insert(0, ROOT)
        from oracle import sde as OS
        self.o = OS.IRSDE(50, self.T, "cosine", 0.005)
        self.image_offset = 0

    def set_mu(self, mu):
        self.mu = mu

    def _z(self, j, tag):
        from daclip_amd import synth
        return synth.synth_noise((1,) + tuple(self.mu.shape[1:]), seed=3000 + self.image_offset + j, tag=tag)

    def noise_state(self, lq):
        out = [self.o.noise_state(lq[j:j + 1].numpy(), self._z(j, "ns")) for j in range(lq.shape[0])]
        return torch.from_numpy(np.concatenate(out or [lq.numpy()[:0]]))

    def reverse_posterior(self, x, text_context, image_context):
        res = []
        for j in range(x.shape[0]):
            mu = self.mu[j:j + 1].numpy()
            self.o.mu = mu
            xj = x[j:j + 1].numpy()
            c = float(text_context[j, 0] - image_context[j, 0])
            for i, t in enumerate(range(self.T, 0, -1)):
                eps = np.tanh(3.0 * (xj - mu) + c).astype(np.float32)
                xj = self.o.posterior_step(xj, eps, t, self._z(j, f"z{i}"))
            res.append(np.ascontiguousarray(xj, np.float32))
        return torch.from_numpy(np.concatenate(res or [x.numpy()[:0]]))


def _run(ws, rank, batch, R):
    import bench
    n_glob, lo, lq, img = bench.shard_inputs(batch, R, ws, rank, "cpu")
    step = bench.make_step(_Clip(), _SDE(), lq, img, lo, n_glob, ws)
    out, el = bench.timed_steps(step, 1, 2, ws, "cpu")
    return n_glob, lo, lq, out, el


def _worker(rank, ws, port, batch, R, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        n_glob, lo, lq, out, el = _run(ws, rank, batch, R)
        q.put((rank, n_glob, lo, lq.numpy(), out.numpy(), el))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_bench_step_sharded_equals_single_rank(ws):
    batch, R = 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, batch, R, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # The same global batch restored by one rank (no collective).
    sys.path[:0] = [ROOT]
    import bench
    n1, lo1, lq1, img1 = bench.shard_inputs(ws * batch, R, 1, 0, "cpu")
    step = bench.make_step(_Clip(), _SDE(), lq1, img1, lo1, n1, 1)
    ref = step().numpy()
    assert ref.shape == (ws * batch, 3, R, R) and np.isfinite(ref).all()
    els = []
    for rank, n_glob, lo, lq, out, el in res:
        assert n_glob == ws * batch and lo == rank * batch
        assert np.array_equal(lq, lq1.numpy()[lo:lo + batch]), f"rank {rank}: shard inputs are not global-indexed"
        assert np.array_equal(out, ref), f"rank {rank}: gathered restore differs from the single-rank one"
        els.append(el)
    assert min(els) > 0 and max(els) == min(els), f"timed_steps must report the max over ranks: {els}"


def _bench(argv, env_extra=None, timeout=240):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                          "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` (the driver's documented form, no launcher around it) starts
    two ranks itself; n_gpus is the process group's world size and both ranks' shards arrive
    in the all-gather (gloo dry run: the same launcher and rank wiring, no GPU)."""
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    js = lines[0]
    assert js["n_gpus"] == 2 and js["ranks_seen"] == [0, 1] and js["global_batch"] == 6
    assert js["steps"] == 2 and js["warmup"] == 1


def test_bench_world_size_must_match_gpus():
    """Under a launcher, WORLD_SIZE != --gpus is an error (never a silent 1-GPU run)."""
    r = _bench(["--gpus", "2", "--dry-run"], dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in (r.stderr + r.stdout)
    r = _bench(["--gpus", "1", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
