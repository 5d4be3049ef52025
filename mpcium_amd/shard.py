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


def safe_primes_sharded(num: int, rank: int, world: int, batch_fn: Callable[[int], List[Tuple[int, int, int]]],
                        max_rounds: int = 1 << 20, gather_every: int = 4, stats: dict | None = None):
    """Config-3 safe-prime search sharded over `world` GPUs:
    rank g tests stream batches b = r*world + g in round r (batch_fn(b) ->
    [(p, q, stream index)] accepted in batch b, e.g. host.safe_prime_batch).
    The ranks exchange their (tiny) lists of accepted primes with ONE
    all-gather per group of R rounds (round 4: one per round, an 8-rank host
    sync per batch): R starts at 1 and then covers the rounds the observed
    acceptance rate says are still needed, capped at `gather_every`. Once
    `num` are known after a gather, every batch below that group's end has
    been tested by some rank, so the `num` smallest stream indices are exactly
    what a single-GPU, stream-order search returns (tss-lib at concurrency 1).
    The only exchange is that host-side gather of a few integers; no
    collective touches the candidate data. Returns the same list on every
    rank; stats (optional dict) receives "rounds" and "gathers"."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    found: List[Tuple[int, int, int]] = []
    r, gathers, R = 0, 0, 1
    while r < max_rounds:
        mine: List[Tuple[int, int, int]] = []
        for k in range(min(R, max_rounds - r)):
            mine.extend(batch_fn((r + k) * world + rank))
        r += min(R, max_rounds - r)
        if world == 1:
            parts = [mine]
        else:
            import torch.distributed as dist
            parts = [None] * world
            dist.all_gather_object(parts, mine)
        gathers += 1
        for p in parts:
            found.extend(p)
        if len(found) >= num:
            found.sort(key=lambda t: t[2])
            if stats is not None:
                stats.update(rounds=r, gathers=gathers)
            return found[:num]
        # every rank sees the same `found` and `r`: the same next R everywhere
        per_round = len(found) / r
        need = num - len(found)
        R = max(1, min(gather_every, -(-need // per_round) if per_round > 0 else gather_every))
        R = int(R)
    raise RuntimeError("safe prime search exhausted max_rounds")
