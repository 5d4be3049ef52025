"""Independent-operand sharding across GPUs (one process per GPU).

The hot path has no exchange step: operands are partitioned into
contiguous per-rank ranges, each rank runs its shard through its own
libmpcx device, and results come back by a host-side gather. No RCCL
collective touches the data path; torch.distributed (gloo) is used only for
the gather of results to one rank and for timing reductions.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple


def shard_range(count: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of `count` operands for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(count, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def run_sharded(fn: Callable[[Sequence], List], items: Sequence, rank: int, world: int,
                gather_to: int = 0):
    """fn(shard) on this rank's shard; the full result list on `gather_to`, None elsewhere."""
    lo, hi = shard_range(len(items), rank, world)
    part = list(fn(items[lo:hi]))
    if world == 1:
        return part
    import torch.distributed as dist
    parts = [None] * world if rank == gather_to else None
    dist.gather_object(part, parts, dst=gather_to)
    if rank != gather_to:
        return None
    out = []
    for p in parts:
        out.extend(p)
    return out


def max_over_ranks(values: Sequence[float], world: int) -> List[float]:
    """Element-wise MAX over ranks (bench timing: the slowest rank defines the step)."""
    if world == 1:
        return list(values)
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]
