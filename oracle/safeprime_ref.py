"""ORACLE -- TEST INFRASTRUCTURE ONLY (see gomath.py header for the import rule).

Restatement of tss-lib v2.0.2 ``common.GetRandomSafePrimesConcurrent`` /
``runGenPrimeRoutine`` (up:common/safe_prime.go; module pinned at
/root/reference/go.mod:10; restated in SURVEY.md 8(a) row A12), run at
concurrency 1 so the first accepted candidate in stream order is the output.

Per candidate:
 1. read (qBitLen+7)/8 bytes from the random source;
 2. bytes[0] &= (1<<b)-1 with b = qBitLen % 8 (8 if 0); set the top two bits
    (bytes[0] |= 3 << (b-2)); make odd (bytes[-1] |= 1);
 3. delta-walk q += delta (delta even, < 2^20) until q mod every small prime
    in {3..53} is non-zero (the walk of Go's old crypto/rand.Prime);
 4. p = 2q + 1; accept iff q has exactly qBitLen bits, 2^(p-1) mod p == 1
    (isPocklingtonCriterionSatisfied) and q is prime (ProbablyPrime(20)).
The acceptance tests are exact up to the (negligible) MR error, so the order
in which they are applied does not change which candidate is accepted first;
extra trial division here only speeds the search up.
"""
from __future__ import annotations

from .gomath import CounterDRBG

SMALL_PRIMES = [3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53]
SMALL_PRIMES_PRODUCT = 16294579238595022365

_TRIAL = [p for p in range(3, 2000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


def miller_rabin(n: int, rounds: int, drbg_seed: int = 0x4D52) -> bool:
    if n < 2:
        return False
    for sp in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % sp == 0:
            return n == sp
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    rng = CounterDRBG(drbg_seed ^ (n & 0xFFFFFFFF))
    bases = [2] + [2 + rng.randbelow(n - 3) for _ in range(rounds)]
    for a in bases:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def candidate_from_bytes(raw: bytes, q_bitlen: int) -> int:
    """Steps 1-3: masking and delta walk. Returns the sieved q (may be 1 bit too long)."""
    b = q_bitlen % 8
    if b == 0:
        b = 8
    bs = bytearray(raw)
    bs[0] &= (1 << b) - 1
    if b >= 2:
        bs[0] |= 3 << (b - 2)
    else:
        bs[0] |= 1
        if len(bs) > 1:
            bs[1] |= 0x80
    bs[-1] |= 1
    q = int.from_bytes(bytes(bs), "big")
    mod = q % SMALL_PRIMES_PRODUCT
    for delta in range(0, 1 << 20, 2):
        m = mod + delta
        if any(m % sp == 0 and (q_bitlen > 6 or m != sp) for sp in SMALL_PRIMES):
            continue
        return q + delta
    return q


def is_safe_prime_pair(q: int, q_bitlen: int) -> bool:
    if q.bit_length() != q_bitlen:
        return False
    p = 2 * q + 1
    for sp in _TRIAL:
        if (q % sp == 0 and q != sp) or (p % sp == 0 and p != sp):
            return False
    if pow(2, p - 1, p) != 1:
        return False
    return miller_rabin(q, 20)


def candidate_stream(seed: int, p_bitlen: int):
    """Yields (index, q) for the deterministic candidate stream (one goroutine)."""
    q_bitlen = p_bitlen - 1
    nbytes = (q_bitlen + 7) // 8
    rng = CounterDRBG(seed)
    idx = 0
    while True:
        yield idx, candidate_from_bytes(rng.read(nbytes), q_bitlen)
        idx += 1


def first_safe_primes(seed: int, p_bitlen: int, num: int, max_candidates: int = 10 ** 7):
    """First `num` safe primes p = 2q+1 of the stream, with their candidate indices."""
    q_bitlen = p_bitlen - 1
    out = []
    for idx, q in candidate_stream(seed, p_bitlen):
        if idx >= max_candidates:
            break
        if is_safe_prime_pair(q, q_bitlen):
            out.append((idx, 2 * q + 1, q))
            if len(out) == num:
                break
    return out
