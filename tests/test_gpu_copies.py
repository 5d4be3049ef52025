"""GPU tests of libmpcx's host-copy rules: pageable
caller buffers are bounced through the lanes' pinned buffers by libmpcx
itself, mpcx_host_alloc blocks are DMA'd directly, a range that starts in a
pinned block and runs past its end is rejected with MPCX_EINVAL before any
copy, and results are identical either way."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pinned(gpu, nwords):
    p = ctypes.c_void_p()
    gpu._check(gpu.lib().mpcx_host_alloc(nwords * 4, ctypes.byref(p)))
    arr = np.ctypeslib.as_array((ctypes.c_uint32 * nwords).from_address(p.value))
    return p, arr


def test_pageable_and_pinned_give_identical_results(gpu, paillier_key):
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    rng = random.Random(55)
    count, w = 300, mod.class_words
    xs = [rng.randrange(N2) for _ in range(count)]
    ys = [rng.getrandbits(700) | 1 for _ in range(count)]
    B = gpu.ints_to_words(xs, w)
    E = gpu.ints_to_words(ys, 22)
    s0 = gpu.copy_stats()
    ref = mod.exp_words(B, E, False, mod.words)  # numpy (pageable) buffers
    s1 = gpu.copy_stats()
    assert s1["bounced_bytes"] - s0["bounced_bytes"] >= B.nbytes + E.nbytes + ref.nbytes
    pb, bp = _pinned(gpu, count * w)
    pe, ep = _pinned(gpu, count * 22)
    po, op = _pinned(gpu, count * mod.words)
    try:
        bp[:] = B.reshape(-1)
        ep[:] = E.reshape(-1)
        gpu._check(gpu.lib().mpcx_modexp_batch(mod.handle, count, pb, w, pe, 22, 0, po, mod.words))
        s2 = gpu.copy_stats()
        assert s2["direct_bytes"] - s1["direct_bytes"] >= B.nbytes + E.nbytes + ref.nbytes
        assert np.array_equal(op.reshape(count, mod.words), ref)
        assert gpu.words_to_ints(ref) == [pow(x, y, N2) for x, y in zip(xs, ys)]
        # a range that starts inside a pinned block and runs past its end
        with pytest.raises(gpu.MpcxError) as ei:
            gpu._check(gpu.lib().mpcx_modexp_batch(mod.handle, count + 1, pb, w, pe, 22, 0, po, mod.words))
        assert ei.value.code == gpu.MPCX_EINVAL
        assert "overruns its pinned allocation" in str(ei.value)
    finally:
        for p in (pb, pe, po):
            gpu._check(gpu.lib().mpcx_host_free(p))
    mod.release()


def test_multi_batch_segment_tables_and_outputs_bounced(gpu, paillier_key):
    """mpcx_modexp_multi_batch with pageable groups: its own segment tables and
    every group's results go through the lane's pinned buffers; results
    equal pow()."""
    N = paillier_key["N"]
    rng = random.Random(7)
    groups = []
    for m in (N, N * N):
        mod = gpu.Modulus(m)
        xs = [rng.randrange(m) for _ in range(rng.randrange(1, 70))]
        ys = [rng.getrandbits(300) | 1 for _ in xs]
        groups.append((mod, xs, ys))
    for mod, xs, ys in groups:  # one class per launch: each group alone, then two groups of one class
        got = gpu.modexp_multi([(mod, xs, ys, None)])
        assert got == [[pow(x, y, mod.m) for x, y in zip(xs, ys)]]
    mod = groups[0][0]
    xs2 = [rng.randrange(N) for _ in range(33)]
    got = gpu.modexp_multi([(mod, groups[0][1], groups[0][2], None), (mod, xs2, 65537, None)])
    assert got[0] == [pow(x, y, N) for x, y in zip(groups[0][1], groups[0][2])]
    assert got[1] == [pow(x, 65537, N) for x in xs2]
