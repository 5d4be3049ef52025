"""Go math/rand (go1.23.5, the generator math/big's ProbablyPrime draws its
Miller-Rabin bases from) -- TEST INFRASTRUCTURE ONLY: restated so the tests
can check the product's Miller-Rabin bases against Go's; nothing under
mpcium_amd/ imports this file.

Restated (go:src/math/rand/rng.go, rng_cooked via go:src/math/rand/gen_cooked.go,
go:src/math/rand/rand.go, go:src/math/big/nat.go nat.random,
go:src/math/big/prime.go probablyPrimeMillerRabin):

* rngSource: additive lagged Fibonacci generator over Z/2^64,
  s_t = s_(t-607) + s_(t-273), held in a 607-word ring (tap, feed pointers).
* Seed(seed): seed mod (2^31 - 1) (0 -> 89482311), the Park-Miller stream
  x <- 48271 x mod (2^31 - 1) run 20 steps, then per ring word three draws
  combined as x0 << 40 ^ x1 << 20 ^ x2, XORed with rngCooked[i].
* rngCooked: the ring of gen_cooked.go's generator (the same ring filled by
  Park-Miller from seed 1 with shifts 20 / 10) after 7.8e12 steps. The
  recurrence is linear, so the 7.8e12 steps are taken here as a jump: x^M mod
  the characteristic polynomial x^607 - x^334 - 1, by square-and-multiply.
* Uint64 / Int63 / Uint32 (Int63 >> 31), nat.random(rand, limit, bitlen):
  64-bit words, each Uint32() | Uint32() << 32, top word masked, retried
  until < limit.

Pinned by Go's documented outputs for seed 1 (tests/test_primes_cpu.py):
Int63() = 5577006791947779410, 8674665223082153551, ... and the Go tour's
rand.Intn(100) sequence 81 87 47 59 81 18 25 40 56 0.
"""
from __future__ import annotations

from functools import lru_cache
from typing import List

import numpy as np

LEN = 607
TAP = 273
M64 = (1 << 64) - 1
MASK63 = (1 << 63) - 1
INT32MAX = (1 << 31) - 1
COOK_STEPS = 7_800_000_000_000


def seedrand(x: int) -> int:
    """x[n+1] = 48271 x[n] mod (2^31 - 1) (Schrage, as rng.go)."""
    hi, lo = divmod(x, 44488)  # x > 0 here
    x = 48271 * lo - 3399 * hi
    if x < 0:
        x += INT32MAX
    return x


def _polymulmod(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """a * b mod (x^607 - x^334 - 1) over Z/2^64 (uint64 arithmetic wraps)."""
    prod = np.zeros(2 * LEN - 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in np.nonzero(a)[0]:
            prod[i:i + LEN] += a[i] * b
        # fold from the top: x^k = x^(k-273) + x^(k-607) for k >= 607
        for k in range(2 * LEN - 2, LEN - 1, -1):
            c = prod[k]
            if c:
                prod[k - TAP] += c
                prod[k - LEN] += c
    return prod[:LEN].copy()


def _xpow(n: int) -> np.ndarray:
    """x^n mod the characteristic polynomial."""
    result = np.zeros(LEN, dtype=np.uint64)
    result[0] = 1
    base = np.zeros(LEN, dtype=np.uint64)
    base[1] = 1
    while n:
        if n & 1:
            result = _polymulmod(result, base)
        n >>= 1
        if n:
            base = _polymulmod(base, base)
    return result


def _ring_to_seq(vec: List[int]) -> List[int]:
    """Ring state (tap = 0, feed = 334, before the next step) as the sequence
    window u_0..u_606 = s_(-607)..s_(-1): step t writes ring position
    (333 - t) mod 607, which holds s_(t-607)."""
    return [vec[(333 - i) % LEN] for i in range(LEN)]


@lru_cache(maxsize=1)
def rng_cooked() -> tuple:
    """rngCooked[607] (int64 values as Go stores them)."""
    # gen_cooked.go srand(1): Park-Miller from seed 1, 20 warm-up steps, then
    # per word x0 << 20 ^ x1 << 10 ^ x2 (no cooked XOR); tap = 0, feed = 334
    x = 1
    vec = [0] * LEN
    for i in range(-20, LEN):
        x = seedrand(x)
        if i >= 0:
            u = x << 20
            x = seedrand(x)
            u ^= x << 10
            x = seedrand(x)
            u ^= x
            vec[i] = u & M64
    u0 = np.array(_ring_to_seq(vec), dtype=np.uint64)
    # window after COOK_STEPS steps: u_(M+i) = sum_k c_k u_(k+i), c = x^M mod P
    c = _xpow(COOK_STEPS)
    out = []
    with np.errstate(over="ignore"):
        ext = list(u0)
        for i in range(LEN):  # extend u0 by the recurrence to u_0 .. u_1213
            ext.append((int(ext[-LEN]) + int(ext[-TAP])) & M64)
        ext = np.array(ext, dtype=np.uint64)
        for i in range(LEN):
            out.append(int(np.sum(c * ext[i:i + LEN], dtype=np.uint64)))
    # step t wrote ring position (333 - t) mod 607; out[i] = s_(M - 607 + i)
    ring = [0] * LEN
    for i in range(LEN):
        ring[(333 - (COOK_STEPS - LEN + i)) % LEN] = out[i]
    return tuple(v - (1 << 64) if v >> 63 else v for v in ring)


class Rand:
    """rand.New(rand.NewSource(seed)) of go1.23.5 math/rand."""

    def __init__(self, seed: int):
        cooked = rng_cooked()
        self.tap = 0
        self.feed = LEN - TAP
        seed %= INT32MAX  # Go: seed % int32max, then + int32max if negative
        if seed == 0:
            seed = 89482311
        x = seed
        self.vec = [0] * LEN
        for i in range(-20, LEN):
            x = seedrand(x)
            if i >= 0:
                u = (x << 40) & M64
                x = seedrand(x)
                u ^= x << 20
                x = seedrand(x)
                u ^= x
                u ^= cooked[i] & M64
                self.vec[i] = u & M64

    def uint64(self) -> int:
        self.tap = (self.tap - 1) % LEN
        self.feed = (self.feed - 1) % LEN
        x = (self.vec[self.feed] + self.vec[self.tap]) & M64
        self.vec[self.feed] = x
        return x

    def int63(self) -> int:
        return self.uint64() & MASK63

    def uint32(self) -> int:
        return self.int63() >> 31

    def int31(self) -> int:
        return self.int63() >> 32

    def int31n(self, n: int) -> int:
        if n & (n - 1) == 0:
            return self.int31() & (n - 1)
        mx = INT32MAX - ((1 << 31) % n)
        v = self.int31()
        while v > mx:
            v = self.int31()
        return v % n

    def intn(self, n: int) -> int:
        """Rand.Intn for 0 < n <= 2^31 - 1."""
        return self.int31n(n)


def nat_random(r: Rand, limit: int) -> int:
    """nat.random(rand, limit, limit.BitLen()) with 64-bit Words: a uniform
    integer in [0, limit)."""
    n = limit.bit_length()
    words = (n + 63) // 64
    msw_bits = n % 64 or 64
    mask = (1 << msw_bits) - 1
    while True:
        z = 0
        for i in range(words):
            w = r.uint32() | (r.uint32() << 32)
            if i == words - 1:
                w &= mask
            z |= w << (64 * i)
        if z < limit:
            return z


def mr_bases(n: int, reps: int) -> List[int]:
    """The Miller-Rabin bases probablyPrimeMillerRabin(reps + 1, force2 = true)
    tries for an odd n > 3 (ProbablyPrime(reps)): reps bases x in [2, n - 2]
    from rand.New(rand.NewSource(int64(n[0]))) (n[0] = the low 64-bit Word,
    as int64), then base 2 last."""
    low = n & M64
    r = Rand(low - (1 << 64) if low >> 63 else low)  # int64(n[0])
    nm3 = n - 3
    out = []
    for _ in range(reps):
        out.append(nat_random(r, nm3) + 2)
    out.append(2)
    return out
