"""Data-parallel sharding of independent restorations over the GPUs of one node.

Every LQ image's encode + T-step reverse loop is independent of every other image
(DenoisingUNet_arch.py:118-174 and sde_utils.py:297-313 have no cross-image term), so a batch
is split into contiguous per-rank shards with no collective on the data path. Only two
collectives exist, both outside the per-step loop:

  * `broadcast_state`: rank 0 owns the state_dicts; one flat RCCL broadcast per network
    replicates them over xGMI (one checkpoint read per node);
  * `gather_outputs`: one all-gather of the restored [b_r,3,H,W] tensors; shards may be
    uneven (B % world != 0), so each rank pads to the largest shard and the padding is cut
    away after the gather.

Device noise is keyed by GLOBAL image index (IRSDE.image_offset -> dac_set_noise_offset), so
a sharded run restores every image bit-identically to an unsharded one. All functions also
run on the gloo backend with CPU tensors (the multi-process tests do that).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_bounds(n: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split: the first n % world ranks get one extra image."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} of {world_size}")
    base, extra = divmod(n, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_sizes(n: int, world_size: int) -> List[int]:
    return [hi - lo for lo, hi in (shard_bounds(n, world_size, r) for r in range(world_size))]


def broadcast_state(sd: Optional[Mapping[str, object]], keys: Sequence[str], device,
                    src: int = 0) -> Dict[str, torch.Tensor]:
    """Replicate rank `src`'s state_dict (values: tensors or arrays) as fp32 views of one flat
    buffer on `device`. Other ranks pass sd=None; shapes travel as a pickled object list."""
    ws, rank = world()
    shapes = [tuple(np.shape(sd[k])) for k in keys] if rank == src else None
    if ws > 1:
        obj = [shapes]
        dist.broadcast_object_list(obj, src=src)
        shapes = obj[0]
    sizes = [int(np.prod(s)) for s in shapes]
    flat = torch.empty(sum(sizes), dtype=torch.float32, device=device)
    if rank == src:
        o = 0
        for k, n in zip(keys, sizes):
            v = sd[k]
            v = v.detach().reshape(-1) if isinstance(v, torch.Tensor) else torch.from_numpy(
                np.ascontiguousarray(v, np.float32).reshape(-1))
            flat[o:o + n].copy_(v.to(torch.float32))
            o += n
    if ws > 1:
        dist.broadcast(flat, src=src)
    out, o = {}, 0
    for k, s, n in zip(keys, shapes, sizes):
        out[k] = flat[o:o + n].view(s)
        o += n
    return out


def gather_outputs(local: torch.Tensor, n_total: int) -> torch.Tensor:
    """All-gather per-rank shards [b_r, ...] (b_r from shard_bounds) into [n_total, ...] on
    every rank, in global image order."""
    ws, rank = world()
    sizes = shard_sizes(n_total, ws)
    if local.shape[0] != sizes[rank]:
        raise RuntimeError(f"rank {rank}: shard has {local.shape[0]} images, expected {sizes[rank]}")
    if ws == 1:
        return local
    m = max(sizes)
    pad = local
    if local.shape[0] < m:
        pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad.contiguous())
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)


def restore_sharded(restore: Callable[[torch.Tensor, int], torch.Tensor], lq: torch.Tensor,
                    gather: bool = True) -> torch.Tensor:
    """Run `restore(lq_shard, first_global_index)` on this rank's contiguous shard of the
    global batch `lq` [B,...] and (optionally) all-gather the restored batch."""
    ws, rank = world()
    lo, hi = shard_bounds(lq.shape[0], ws, rank)
    # A rank with an empty shard (B < world) still joins the gather; restored images have
    # the LQ shape, so its empty contribution is an empty slice of lq.
    out = restore(lq[lo:hi], lo) if hi > lo else lq[lo:hi].clone()
    return gather_outputs(out, lq.shape[0]) if gather else out
