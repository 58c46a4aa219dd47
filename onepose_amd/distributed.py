"""Frame-sharded multi-GPU execution.

Frames are independent given the object, so a batch of query frames shards contiguously over
ranks (one process per GPU, ``torch.distributed`` over RCCL; gloo on CPU for tests).  Each
rank holds its own replica of the packed weights and the object and runs its frames with no
data-path collective; the only exchange is one all-gather of the small per-frame result rows
(pose, errors, cm/deg flags: ~150 B per frame).  The reference processes frames one by one
on a single device (``inference.py:132-177``); this is the build's scale-out, not a port.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env():
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 when absent)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl", device=None):
    """Join the process group when WORLD_SIZE > 1 (MASTER_ADDR/PORT from the environment).
    Returns True when a group is active.  ONEPOSE_FORCE_PG=1 (diagnostic, under
    torch.distributed.run) joins it at WORLD_SIZE 1 too, so that a one-GPU box runs the N > 1
    bench path with its RCCL communicator and streams."""
    world, _, _ = env()
    if world <= 1 and not (os.environ.get("ONEPOSE_FORCE_PG") == "1"
                           and "MASTER_ADDR" in os.environ):
        return False
    if not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return True


def frame_shard(n_frames: int, world: int, rank: int):
    """Contiguous [start, stop) of `n_frames` owned by `rank`: ceil(n/world) per rank, the
    last ranks possibly short or empty."""
    per = -(-n_frames // world) if world > 0 else n_frames
    start = min(rank * per, n_frames)
    return start, min(start + per, n_frames)


def gather_frames(local: torch.Tensor, n_frames: int, group=None) -> torch.Tensor:
    """All-gather per-frame result rows ([n_local, F], rank order = frame order) into the
    full [n_frames, F] on every rank.  Shards are padded to the common ceil size so one
    collective suffices; the padding is dropped after."""
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size(group)
    per = -(-n_frames // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    rows = []
    for r in range(world):
        s, e = frame_shard(n_frames, world, r)
        rows.append(parts[r][:e - s])
    return torch.cat(rows, 0)


def max_over_ranks(x: float, device=None) -> float:
    """Max of a host scalar over ranks (the bench's timed region: slowest rank)."""
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
