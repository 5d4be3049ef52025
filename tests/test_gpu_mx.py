"""k_modexp_mx -- the 4096-bit main geometry with its Montgomery reduction on the
i8 matrix cores (mpcium_amd/csrc/mpcx_mx.hpp) -- against Python's pow and against
the CIOS kernel (k_modexp) on the same inputs: bit-exact.

The shapes follow the reference's hot path: r^N mod N^2 with a shared 2048-bit N
(config 2, up:crypto/paillier Encrypt), per-operand exponents (HomoMult c^m), a
multiplier (Encrypt's Gamma^m * r^N), and the edge operands 0, 1, m - 1.
"""
import random

import pytest

from mpcium_amd import mpcx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    mpcx.init(0)
    keys = ("mx", "geom_policy")
    saved = {k: mpcx.get_option(k) for k in keys}  # the later test modules see the defaults again
    mpcx.set_option("kernel_stats", 1)
    mpcx.set_option("geom_policy", 2)  # the main geometry at every batch size
    yield
    for k in keys:
        mpcx.set_option(k, saved[k])
    mpcx.set_option("kernel_stats", 0)


def _modulus(rng, bits=4096):
    # N^2 of a random odd 2048-bit N (top bit set): the Paillier modulus shape
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    return n, n * n


def _run(m, bases, exps, mx, muls=None):
    mpcx.set_option("mx", mx)
    mpcx.kernel_stats(reset=True)
    mod = mpcx.Modulus(m)
    try:
        out = mod.exp_mul(bases, exps, muls) if muls is not None else mod.exp(bases, exps)
    finally:
        mod.release()
    return out, mpcx.kernel_stats()


def _mx_launched(stats, geom=2):
    return any(k.get("kind") == "modexp_mx" and k.get("geom") == geom and k.get("launches", 0) > 0
               for k in stats.get("kernels", []))


def test_mx_shared_exponent_matches_pow_and_cios(dev):
    rng = random.Random(5101)
    n, m = _modulus(rng)
    bases = [rng.randrange(m) for _ in range(4096)]
    bases[0], bases[1], bases[2], bases[3] = 0, 1, m - 1, 2
    got, st = _run(m, bases, n, 1)
    assert _mx_launched(st), st
    ref, st0 = _run(m, bases, n, 0)
    assert not _mx_launched(st0)
    assert got == ref
    for i in list(range(8)) + rng.sample(range(8, len(bases)), 56):
        assert got[i] == pow(bases[i], n, m), i


def test_mx_per_operand_exponents(dev):
    rng = random.Random(5102)
    _, m = _modulus(rng)
    bases = [rng.randrange(m) for _ in range(2048)]
    exps = [rng.getrandbits(rng.choice([1, 2, 64, 256, 2048])) for _ in bases]
    exps[0], exps[1] = 0, 1
    got, st = _run(m, bases, exps, 1)
    assert _mx_launched(st)
    for i in list(range(4)) + rng.sample(range(4, len(bases)), 60):
        assert got[i] == pow(bases[i], exps[i], m), i


def test_mx_with_multiplier(dev):
    rng = random.Random(5103)
    n, m = _modulus(rng)
    bases = [rng.randrange(m) for _ in range(2048)]
    muls = [rng.randrange(m) for _ in bases]
    got, st = _run(m, bases, n, 1, muls=muls)
    assert _mx_launched(st)
    ref, _ = _run(m, bases, n, 0, muls=muls)
    assert got == ref
    for i in rng.sample(range(len(bases)), 32):
        assert got[i] == muls[i] * pow(bases[i], n, m) % m, i


def test_mx_small_exponents_and_odd_moduli(dev):
    # shared exponents of 1..7 bits (short schedules, the odd-power table's
    # restaged rows) and moduli well below 2^4096
    rng = random.Random(5104)
    for bits in (4096, 3001, 2081):
        m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        bases = [rng.randrange(m) for _ in range(2048)]
        for e in (1, 2, 3, 5, 127, (1 << 70) + 12345):
            got, st = _run(m, bases, e, 1)
            assert _mx_launched(st)
            for i in rng.sample(range(len(bases)), 12):
                assert got[i] == pow(bases[i], e, m), (bits, e, i)


def test_mx_2048_geometry5(dev):
    # the 2048-bit class's lane-pair geometry (32 operands per wave, two MFMA halves):
    # ModProof's Z^N mod N shape (shared 2048-bit N), per-operand exponents, a multiplier
    rng = random.Random(5105)
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    bases = [rng.randrange(n) for _ in range(4096)]
    bases[0], bases[1], bases[2] = 0, 1, n - 1
    got, st = _run(n, bases, n, 2)  # mx = 2: the lane-pair geometry too (off by default)
    assert _mx_launched(st, 5), st
    ref, st0 = _run(n, bases, n, 0)
    assert not _mx_launched(st0, 5)
    assert got == ref
    for i in list(range(3)) + rng.sample(range(3, len(bases)), 40):
        assert got[i] == pow(bases[i], n, n), i
    exps = [rng.getrandbits(rng.choice([1, 5, 300, 2048])) for _ in bases]
    got, st = _run(n, bases, exps, 2)
    assert _mx_launched(st, 5)
    for i in rng.sample(range(len(bases)), 40):
        assert got[i] == pow(bases[i], exps[i], n), i
    muls = [rng.randrange(n) for _ in bases]
    got, st = _run(n, bases, 65537, 2, muls=muls)
    assert _mx_launched(st, 5)
    for i in rng.sample(range(len(bases)), 24):
        assert got[i] == muls[i] * pow(bases[i], 65537, n) % n, i
    # moduli below the class maximum (N~ is a product of two 1024-bit safe primes: 2047-2048 bits)
    for bits in (2047, 1800):
        m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        b2 = [rng.randrange(m) for _ in range(2048)]
        got, st = _run(m, b2, 3, 2)
        assert _mx_launched(st, 5)
        for i in rng.sample(range(len(b2)), 16):
            assert got[i] == pow(b2[i], 3, m), (bits, i)


def test_mx_default_leaves_the_lane_pair_geometry_on_cios(dev):
    rng = random.Random(5106)
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    bases = [rng.randrange(n) for _ in range(4096)]
    got, st = _run(n, bases, n, 1)
    assert not _mx_launched(st, 5)
    for i in rng.sample(range(len(bases)), 8):
        assert got[i] == pow(bases[i], n, n)


def test_mx_multi_batch_segments(dev):
    # k_modexp_multi_mx: several 4096-bit moduli in one launch, every segment on a
    # workgroup boundary with its own tables (the shape of signing's and config 1's
    # merged Paillier launches): bit-exact against pow and against k_modexp_multi
    rng = random.Random(5107)
    mods, groups = [], []
    for t, cnt in enumerate((300, 1024, 257, 700)):
        n, m = _modulus(rng)
        mod = mpcx.Modulus(m)
        mods.append(mod)
        bases = [rng.randrange(m) for _ in range(cnt)]
        if t == 0:
            groups.append((mod, bases, n, None))  # shared exponent (Encrypt's r^N)
        elif t == 1:
            groups.append((mod, bases, [rng.getrandbits(256) for _ in bases], None))  # HomoMult c^b
        elif t == 2:
            groups.append((mod, bases, n, [rng.randrange(m) for _ in bases]))  # with a multiplier
        else:
            groups.append((mod, bases, 65537, None))
    try:
        mpcx.set_option("mx", 1)
        mpcx.kernel_stats(reset=True)
        got = mpcx.modexp_multi(groups)
        st = mpcx.kernel_stats()
        assert any(k.get("kind") == "modexp_multi_mx" and k.get("launches", 0) > 0 for k in st["kernels"]), st
        mpcx.set_option("mx", 0)
        ref = mpcx.modexp_multi(groups)
        assert got == ref
        for (mod, bases, exps, muls), out in zip(groups, got):
            m = mod.m
            for i in rng.sample(range(len(bases)), 6):
                e = exps if isinstance(exps, int) else exps[i]
                want = pow(bases[i], e, m)
                if muls is not None:
                    want = want * muls[i] % m
                assert out[i] == want
    finally:
        for mod in mods:
            mod.release()


def test_mx_structured_moduli(dev):
    # moduli whose digit strings stress the reduction's bounds: all-ones (the
    # largest i8 column sums of m and of m'' = 1), one sparse (m = 2^4095 + 1, m'' dense),
    # 2^4096 - 2^2048 - 1 (a long run of ones over zeros), each with bases at the
    # edges (0, 1, 2, m - 1, m - 2) and random ones; shared and per-operand exponents
    rng = random.Random(5108)
    mods = ((1 << 4096) - 1, (1 << 4095) + 1, (1 << 4096) - (1 << 2048) - 1)
    for m in mods:
        bases = [rng.randrange(m) for _ in range(2048)]
        bases[:5] = [0, 1, 2, m - 1, m - 2]
        for e in ((1 << 2048) - 1, rng.getrandbits(2048) | 1):
            got, st = _run(m, bases, e, 1)
            assert _mx_launched(st), st
            for i in list(range(5)) + rng.sample(range(5, len(bases)), 11):
                assert got[i] == pow(bases[i], e, m), (hex(m)[:12], i)
        exps = [rng.getrandbits(rng.choice([1, 17, 256, 4096])) for _ in bases]
        got, st = _run(m, bases, exps, 1)
        assert _mx_launched(st)
        for i in list(range(5)) + rng.sample(range(5, len(bases)), 11):
            assert got[i] == pow(bases[i], exps[i], m), (hex(m)[:12], i)


def test_mx_ragged_batch_unreduced_operands(dev):
    """a single k_modexp_mx launch whose last workgroup has spare
    wavefronts (2,100 operands: not a whole number of MX_WG-wave workgroups of 16
    operands per wave) and bases / multipliers at or above m, up to the class's
    word width (what the C-ABI accepts): bit-exact against pow and the CIOS kernel."""
    rng = random.Random(5109)
    n, m = _modulus(rng)
    mod = mpcx.Modulus(m)
    lim = 1 << (32 * mod.class_words)
    mod.release()
    count = 2100
    bases = [rng.randrange(m, lim) if i % 3 == 0 else rng.randrange(m) for i in range(count)]
    bases[1], bases[2] = lim - 1, m
    muls = [rng.randrange(m, lim) if i % 2 else rng.randrange(m) for i in range(count)]
    got, st = _run(m, bases, n, 1, muls=muls)
    assert _mx_launched(st), st
    ref, st0 = _run(m, bases, n, 0, muls=muls)
    assert not _mx_launched(st0)
    assert got == ref
    for i in list(range(4)) + rng.sample(range(4, count), 28) + [count - 1]:
        assert got[i] == muls[i] * pow(bases[i], n, m) % m, i
    # per-operand exponents on the same ragged batch
    exps = [rng.getrandbits(256) for _ in range(count)]
    got, st = _run(m, bases, exps, 1)
    assert _mx_launched(st)
    for i in [0, 1, 2, count - 1] + rng.sample(range(3, count - 1), 20):
        assert got[i] == pow(bases[i], exps[i], m), i
