"""World-size-2 gloo tests of the multi-GPU sharding plumbing on CPU.
The per-shard compute is a stand-in (CPython pow); on the GPU box each rank
would call libmpcx on its own device."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from mpcium_amd.shard import shard_range


def test_shard_range_partition():
    for count in (0, 1, 7, 9, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(count, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == count
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from mpcium_amd.shard import max_over_ranks, run_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = (1 << 127) - 1
    items = list(range(3, 3 + 101))
    out = run_sharded(lambda xs: [pow(x, 65537, m) for x in xs], items, rank, world)
    t = max_over_ranks([0.5 + rank, 2.0 - rank], world)
    if rank == 0:
        q.put((out == [pow(x, 65537, m) for x in items], t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_and_max_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, t = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert t == [1.5, 2.0]


def _fake_batch(b):
    """Stand-in for host.safe_prime_batch: a deterministic, sparse set of
    'accepted' stream indices per batch of 100 candidates."""
    import random
    rng = random.Random(b)
    return [(2 * i + 3, i + 1, i) for i in sorted(rng.sample(range(b * 100, b * 100 + 100), rng.choice([0, 0, 1, 2])))]


def _sp_worker(rank, world, port, q):
    import torch.distributed as dist
    from mpcium_amd.shard import safe_primes_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = safe_primes_sharded(7, rank, world, _fake_batch)
    st = {}
    big = safe_primes_sharded(40, rank, world, _fake_batch, stats=st)
    q.put((rank, (out, big, st)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_safe_primes_sharded_world2_matches_stream_order():
    from mpcium_amd.shard import safe_primes_sharded
    single = safe_primes_sharded(7, 0, 1, _fake_batch)
    assert [t[2] for t in single] == sorted(t[2] for t in single) and len(single) == 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    st1 = {}
    big1 = safe_primes_sharded(40, 0, 1, _fake_batch, stats=st1)
    for r in (0, 1):
        out, big, st = res[r]
        assert out == single
        # batched gathers (one per group of rounds): the same stream-order result
        assert big == big1 and [t[2] for t in big] == sorted(t[2] for t in big) and len(big) == 40
        assert st["gathers"] < st["rounds"], st
