"""CPU tests of the primality oracle (oracle/safeprime_ref.py), pinned against
published integer sequences:

* the extra strong Lucas pseudoprimes (OEIS A217719: the composites that Go's
  math/big probablyPrimeLucas accepts) below 80,000;
* the strong pseudoprimes to base 2 (OEIS A001262) below 100,000 -- the
  composites one Miller-Rabin round with base 2 accepts;
* ProbablyPrime == trial-division primality for 64 <= n < 20,000, and known
  large primes / BPSW-exercising composites.
"""
import math

from oracle import safeprime_ref as S

A217719 = [989, 3239, 5777, 10877, 27971, 29681, 30739, 31631, 39059, 72389, 73919, 75077]
A001262 = [2047, 3277, 4033, 4681, 8321, 15841, 29341, 42799, 49141, 52633, 65281, 74665, 80581, 85489, 88357,
           90751]


def _composite(n):
    return any(n % d == 0 for d in range(2, math.isqrt(n) + 1))


def test_lucas_pseudoprimes_match_a217719():
    got = [n for n in range(5, 80000, 2) if S.probably_prime_lucas(n) and _composite(n)]
    assert got == A217719


def test_base2_strong_pseudoprimes_match_a001262():
    got = [n for n in range(5, 100000, 2) if S.strong_probable_prime(n, 2) and _composite(n)]
    assert got == A001262


def test_probably_prime_small_range():
    for n in range(0, 20000):
        assert S.probably_prime(n) == (n > 1 and not _composite(n)), n


def test_probably_prime_large():
    for e in (521, 607, 1279):  # Mersenne primes
        assert S.probably_prime((1 << e) - 1)
    # strong pseudoprime to bases 2..23 (= 149491 * 747451 * 34233211): the Lucas step rejects it
    n = 3825123056546413051
    assert n == 149491 * 747451 * 34233211
    assert all(S.strong_probable_prime(n, a) for a in (2, 3, 5, 7, 11, 13, 17, 19, 23))
    assert not S.probably_prime_lucas(n) and not S.probably_prime(n)
    assert not S.probably_prime(((1 << 521) - 1) * ((1 << 607) - 1))


def test_lucas_param_exits():
    """Baillie-OEIS method C: Jacobi(P^2-4, n) = -1 runs the test; = 0 means
    P+2 | n (prime iff n == P+2); squares never reach -1 (checked at P = 40)."""
    assert S.lucas_param(7) == (1, 3)       # (5/7) = -1
    assert S.lucas_param(5) == (2, None)    # (5/5) = 0 and 5 == 3 + 2
    assert S.lucas_param(25) == (0, None)   # (5/25) = 0, 25 != 5
    assert S.lucas_param(9) == (0, None)    # (5/9) = 1, (12/9) = 0
    assert S.lucas_param(10007 ** 2) == (0, None)  # square: caught at P = 40


# Go's documented math/rand outputs for rand.New(rand.NewSource(1)): the first
# Int63() values, and the Go tour's rand.Intn(100) sequence.
GO_SEED1_INT63 = [5577006791947779410, 8674665223082153551, 6129484611666145821]
GO_TOUR_INTN100 = [81, 87, 47, 59, 81, 18, 25, 40, 56, 0]


def test_go_rand_oracle_pinned_by_documented_outputs():
    from oracle import gorand as G
    r = G.Rand(1)
    assert [r.int63() for _ in range(3)] == GO_SEED1_INT63
    r = G.Rand(1)
    assert [r.intn(100) for _ in range(10)] == GO_TOUR_INTN100


def test_go_rand_product_matches_oracle():
    """libmpcx_host's Go math/rand (csrc/host/gorand.cpp): the documented
    seed-1 outputs, other seeds (negative, 0, above 2^31) and ProbablyPrime's
    Miller-Rabin bases against the oracle."""
    import random
    from mpcium_amd import host
    from oracle import gorand as G
    assert host.go_rand_int63(1, 3) == GO_SEED1_INT63
    for seed in (0, -1, 7, 2 ** 31 - 1, 2 ** 31, -(2 ** 63), 2 ** 63 - 1, 0x5DEECE66D):
        r = G.Rand(seed)
        assert host.go_rand_int63(seed, 700) == [r.int63() for _ in range(700)], seed
    rng = random.Random(5)
    for bits in (67, 128, 1024, 1025, 2048):
        for _ in range(3):
            n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
            assert host.go_mr_bases(n, 20) == G.mr_bases(n, 20)[:-1], (bits, n)
            assert all(2 <= b <= n - 2 for b in G.mr_bases(n, 20))
