"""Host-side big-integer helpers of libmpcx_host on CPU (no GPU): the batched
coprimality test (mpcxh_coprime_batch, the gcd behind
common.GetRandomPositiveRelativelyPrimeInt and the proof verifiers' gcd
checks) against math.gcd, including shared factors, x >= m, x = 0, and
operand sizes from one word to 4096 bits (the N^2 class)."""
import math
import random

import pytest


@pytest.fixture(scope="module")
def host():
    from mpcium_amd import build, host
    build.build()
    return host


def _odd(rng, bits):
    return rng.getrandbits(bits) | (1 << (bits - 1)) | 1


@pytest.mark.parametrize("bits", [5, 63, 64, 65, 127, 200, 1024, 2048, 4096])
def test_coprime_matches_gcd(host, bits):
    rng = random.Random(bits)
    xs, ms = [], []
    for k in range(96):
        m = _odd(rng, bits)
        if k % 4 == 0:      # shared odd factor
            f = _odd(rng, max(2, bits // 3))
            m = (m // f) * f | 1
            if m % f:
                m = f * _odd(rng, max(2, bits - f.bit_length()))
            x = f * rng.getrandbits(max(1, bits - f.bit_length()))
        elif k % 4 == 1:    # x >= m, random size
            x = rng.getrandbits(2 * bits)
        elif k % 4 == 2:    # power-of-two multiples of a coprime value
            x = rng.getrandbits(bits) << rng.randrange(0, 70)
        else:
            x = rng.getrandbits(bits)
        xs.append(x)
        ms.append(m)
    xs += [0, 1, ms[0], ms[1] * 3, 2]
    ms += [ms[0], ms[0], ms[0], ms[1], ms[2]]
    want = [math.gcd(x, m) == 1 for x, m in zip(xs, ms)]
    assert host.coprime(xs, ms) == want
    assert any(want) and not all(want)


def test_coprime_safe_prime_products(host):
    """Paillier-shaped moduli: x sharing exactly one prime factor of N = PQ."""
    rng = random.Random(7)
    P = (1 << 1023) + 1155   # odd, not necessarily prime: only the gcd matters
    Q = (1 << 1023) + 3195
    N = P * Q
    xs = [P * rng.getrandbits(900), Q * rng.getrandbits(900), rng.getrandbits(2048), N - 1, N + P]
    assert host.coprime(xs, [N] * len(xs)) == [math.gcd(x, N) == 1 for x in xs]


def test_coprime_rejects_even_modulus(host):
    from mpcium_amd.mpcx import MpcxError
    with pytest.raises(MpcxError):
        host.coprime([3], [10])


def _edge_values(rng, bits):
    """Random values plus the shapes that stress Knuth D on 64-bit limbs:
    all-ones limbs, a lone top bit, odd and even 32-bit word counts."""
    return [rng.getrandbits(bits) | (1 << (bits - 1)), (1 << bits) - 1, 1 << (bits - 1),
            ((1 << bits) - 1) ^ ((1 << (bits // 2)) - 1)]


@pytest.mark.parametrize("abits,bbits", [(32, 32), (64, 31), (96, 64), (128, 65), (256, 256), (520, 130),
                                         (2048, 256), (4096, 2048), (4127, 2049), (8192, 4096), (8190, 4064),
                                         (3072, 1023)])
def test_nat_mul_divmod_match_python(host, abits, bbits):
    """Nat * / % (64-bit limb schoolbook and Knuth D) equal Python's ints,
    including the add-back and the 128-bit trial-quotient corrections."""
    rng = random.Random(abits * 7919 + bbits)
    for a in _edge_values(rng, abits) + [rng.getrandbits(abits) for _ in range(20)]:
        for b in _edge_values(rng, bbits) + [rng.getrandbits(bbits) | 1 for _ in range(5)]:
            if b == 0:
                continue
            assert host.nat_arith(0, a, b) == a * b
            assert host.nat_arith(1, a, b) == a // b
            assert host.nat_arith(2, a, b) == a % b
    # quotient digits that force qhat corrections: u = q v + r with q's limbs at
    # the top of their range and r = v - 1
    for _ in range(50):
        v = rng.getrandbits(bbits) | (1 << (bbits - 1))
        q = (1 << (64 * rng.randint(1, 4))) - rng.randint(1, 3)
        u = q * v + (v - 1)
        assert host.nat_arith(1, u, v) == q
        assert host.nat_arith(2, u, v) == v - 1
    assert host.nat_arith(0, 0, 5) == 0 and host.nat_arith(1, 3, 5) == 0 and host.nat_arith(2, 3, 5) == 3


@pytest.mark.parametrize("bits", [64, 256, 1024, 2048])
def test_nat_modinv_gcd_match_python(host, bits):
    rng = random.Random(bits)
    for _ in range(10):
        m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        x = rng.getrandbits(bits + 7)
        assert host.nat_arith(4, x, m) == math.gcd(x, m)
        if math.gcd(x, m) == 1:
            assert host.nat_arith(3, x, m) == pow(x, -1, m)
        else:
            with pytest.raises(host.MpcxError):
                host.nat_arith(3, x, m)
