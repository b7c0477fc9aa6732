"""Data-parallel pieces of the fused training path (one process per GPU).

The reference trains on one device (training.py:15-64); SURVEY 8(e) /
BASELINE cfg 4 scale it as DistributedDataParallel would: every rank owns a
shard of the pair arrays, keeps LOCAL BatchNorm statistics (no SyncBN), and
the only exchange per step is one all-reduce (average) of the flat fp32
gradient arena -- 85 KB at cfg 3 -- over RCCL/xGMI (``backend="nccl"``) or
gloo (CPU tests).  Parameters start identical on every rank (DDP broadcasts
rank 0's state at construction: ``broadcast_state_``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) of the contiguous shard of ``n`` pairs owned by ``rank``
    (ceil(n / world) per rank, the last one shorter -- DistributedSampler
    without padding)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    per = -(-n // world)
    lo = min(rank * per, n)
    return lo, min(lo + per, n)


def world_of(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def average_gradients_(flat_grad: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean over ranks of the flat gradient arena (one collective)."""
    if not (dist.is_available() and dist.is_initialized()):
        return flat_grad
    w = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":  # RCCL averages inside the collective (no extra kernel)
        dist.all_reduce(flat_grad, op=dist.ReduceOp.AVG, group=group)
        return flat_grad
    dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)
    if w > 1:
        flat_grad.mul_(1.0 / w)
    return flat_grad


def broadcast_state_(params: torch.Tensor, buffers: Optional[torch.Tensor] = None, group=None, src: int = 0):
    """Make every rank start from rank ``src``'s parameters / BN buffers."""
    if world_of(group) > 1:
        dist.broadcast(params, src=src, group=group)
        if buffers is not None:
            dist.broadcast(buffers, src=src, group=group)
