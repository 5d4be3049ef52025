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

Go (*Int).ProbablyPrime(n) (go:src/math/big/prime.go, go1.23.5 per
/root/reference/go.mod:5) is restated as: the x < 64 bitmask, the even and
small-prime (3..53) exits, Miller-Rabin with n+1 rounds whose last base is 2,
then probablyPrimeLucas -- the "extra strong" Lucas test with Baillie-OEIS
method C parameters (P = 3, 4, ... until Jacobi(P^2-4, x) = -1, Q = 1). The
other n Miller-Rabin bases are Go's: math/rand seeded with x's low word
(oracle/gorand.py, pinned by Go's documented seed-1 outputs).

generate_preparams: keygen.GeneratePreParams on ONE stream, searches in a
fixed order (Paillier's 2 safe primes, retried until |P - Q| has >= 1021 bits;
then N~'s 2), each consuming the stream exactly through its last accepted
candidate (tss-lib at concurrency 1), then f and alpha
(GetRandomPositiveRelativelyPrimeInt(N~)), beta = alpha^-1 mod pq,
h1 = f^2 mod N~, h2 = h1^alpha mod N~.
"""
from __future__ import annotations

from . import gorand
from .gomath import CounterDRBG

SMALL_PRIMES = [3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53]
SMALL_PRIMES_PRODUCT = 16294579238595022365

_TRIAL = [p for p in range(3, 2000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


_SMALL_MASK = sum(1 << p for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61))


def mr_bases(n: int, reps: int):
    """Base 2, then Go's `reps` bases in [2, n-2] (oracle/gorand.py; Go runs
    base 2 last, the decision does not depend on the order)."""
    return [2] + gorand.mr_bases(n, reps)[:-1]


_pw = pow  # x^y mod m: hookable (bench.py's CPU legs time Go's expNN restated in C here)


def strong_probable_prime(n: int, a: int) -> bool:
    """One Miller-Rabin round of go:src/math/big/prime.go probablyPrimeMillerRabin."""
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    y = _pw(a, d, n)
    if y in (1, n - 1):
        return True
    for _ in range(1, s):
        y = y * y % n
        if y == n - 1:
            return True
        if y == 1:
            return False
    return False


def jacobi(a: int, n: int) -> int:
    """math/big Jacobi(a, n) for odd n > 0."""
    a %= n
    j = 1
    while a:
        while a % 2 == 0:
            a //= 2
            if n % 8 in (3, 5):
                j = -j
        a, n = n, a
        if a % 4 == 3 and n % 4 == 3:
            j = -j
        a %= n
    return j if n == 1 else 0


def lucas_param(n: int):
    """Baillie-OEIS method C: (1, P) to run the test, (0, None) composite, (2, None) prime."""
    import math
    p = 3
    while True:
        if p > 10000:
            raise RuntimeError("no D with (D/n) = -1")
        j = jacobi(p * p - 4, n)
        if j == -1:
            return 1, p
        if j == 0:
            return (2 if n == p + 2 else 0), None
        if p == 40 and math.isqrt(n) ** 2 == n:
            return 0, None
        p += 1


def probably_prime_lucas(n: int) -> bool:
    """go:src/math/big/prime.go probablyPrimeLucas (extra strong Lucas test)."""
    if n <= 1:
        return False
    if n % 2 == 0:
        return n == 2
    r, P = lucas_param(n)
    if r != 1:
        return r == 2
    s = n + 1
    rr = 0
    while s % 2 == 0:
        s //= 2
        rr += 1
    vk, vk1 = 2, P
    for i in range(s.bit_length(), -1, -1):
        if (s >> i) & 1:
            vk, vk1 = (vk * vk1 - P) % n, (vk1 * vk1 - 2) % n
        else:
            vk1, vk = (vk * vk1 - P) % n, (vk * vk - 2) % n
    if vk in (2, n - 2) and (P * vk - 2 * vk1) % n == 0:
        return True
    for _ in range(rr - 1):
        if vk == 0:
            return True
        if vk == 2:
            return False
        vk = (vk * vk - 2) % n
    return False


def probably_prime(n: int, reps: int = 20) -> bool:
    """go (*Int).ProbablyPrime(reps) decision (see the module header for the bases)."""
    if n < 64:
        return n >= 0 and bool((_SMALL_MASK >> n) & 1)
    if n % 2 == 0:
        return False
    if any(n % p == 0 for p in (3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53)):
        return False
    return all(strong_probable_prime(n, a) for a in mr_bases(n, reps)) and probably_prime_lucas(n)


def miller_rabin(n: int, rounds: int) -> bool:
    """ProbablyPrime(rounds) (kept name for callers)."""
    return probably_prime(n, rounds)


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


def first_safe_primes_from(rng, p_bitlen: int, num: int, max_candidates: int = 10 ** 7):
    """The same search on an open stream `rng` (.read(n)), consuming exactly
    through the num-th accepted candidate -> [(index, p, q)]."""
    q_bitlen = p_bitlen - 1
    nbytes = (q_bitlen + 7) // 8
    out = []
    for idx in range(max_candidates):
        q = candidate_from_bytes(rng.read(nbytes), q_bitlen)
        if is_safe_prime_pair(q, q_bitlen):
            out.append((idx, 2 * q + 1, q))
            if len(out) == num:
                return out
    raise RuntimeError("safe prime search exhausted max_candidates")


def generate_preparams(seed: int):
    """keygen.GeneratePreParams on the CounterDRBG(seed) stream (see header) ->
    dict of the 12 LocalPreParams fields + the stream bytes consumed."""
    from . import tss_ref as T
    rng = CounterDRBG(seed)
    consumed = [0]

    class _R:
        def read(self, n):
            consumed[0] += n
            return rng.read(n)
    r = _R()
    while True:
        sg = first_safe_primes_from(r, 1024, 2)
        P, Q = sg[0][1], sg[1][1]
        if abs(P - Q).bit_length() >= 1024 - 3:
            break
    N = P * Q
    phi = (P - 1) * (Q - 1)
    import math
    lam = phi // math.gcd(P - 1, Q - 1)
    sg = first_safe_primes_from(r, 1024, 2)
    Pt, Qt = sg[0][1], sg[1][1]
    p, q = sg[0][2], sg[1][2]
    NT = Pt * Qt
    f1 = T.get_random_positive_relatively_prime_int(r, NT)
    alpha = T.get_random_positive_relatively_prime_int(r, NT)
    beta = pow(alpha, -1, p * q)
    h1 = f1 * f1 % NT
    h2 = pow(h1, alpha, NT)
    return {"N": N, "LambdaN": lam, "PhiN": phi, "P": P, "Q": Q, "NTildei": NT, "H1i": h1, "H2i": h2,
            "Alpha": alpha, "Beta": beta, "p": p, "q": q, "consumed_bytes": consumed[0]}


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
