"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (mpcium_amd/) never imports it.

Pure-Python restatements of the arithmetic on the reference's hot path:

* ``go_exp(x, y, m)``   -- Go ``(*big.Int).Exp`` (go1.23.5, go:src/math/big/int.go,
  ``Int.exp``) as reached from tss-lib v2.0.2 ``common.ModInt(m).Exp``
  (up:common/int.go; module pinned at /root/reference/go.mod:10).  Sign rules:
  y < 0 -> x is replaced by ModInverse(x, m) (nil if none); the result takes the
  sign of x when y is odd and is then made positive mod |m|.
* Paillier (up:crypto/paillier/paillier.go): encrypt / homo_mult / homo_add /
  decrypt and L(u) = (u-1)/N exactly as SURVEY.md section 8(a) rows A3-A6 restate them.
* Safe-prime candidate stream (up:common/safe_prime.go, runGenPrimeRoutine):
  see safeprime_ref.py.

The modexp core is CPython ``pow`` -- an implementation independent of both the
GPU kernels and the C restatement in gomodexp.c, cross-checked against GMP and
OpenSSL by tests/golden/gen_golden.py.  Parity with the reference itself is
unpinned: Go and tss-lib are absent from this image ("Oracle").
"""
from __future__ import annotations

import hashlib
import math
from typing import Optional

SECP256K1_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def mod_inverse(g: int, n: int) -> Optional[int]:
    """Go (*Int).ModInverse (int.go): inverse of g in Z/|n|Z, None if gcd != 1."""
    n = abs(n)
    if n == 0:
        return None
    g %= n
    if math.gcd(g, n) != 1:
        return None
    if n == 1:
        return 0
    return pow(g, -1, n)


def go_exp(x: int, y: int, m: Optional[int]) -> Optional[int]:
    """Restatement of go1.23.5 (*Int).exp(x, y, m, slow=false), go:src/math/big/int.go.

    Returns None where Go returns nil (y < 0 and x not invertible mod m).
    """
    x_abs, x_neg = abs(x), x < 0
    if y < 0:
        if m is None or m == 0:
            return 1
        inv = mod_inverse(x, m)
        if inv is None:
            return None
        x_abs = inv  # xWords = inverse.abs (x.neg is still consulted below)
    y_abs = abs(y)
    m_abs = abs(m) if m is not None else 0
    if m_abs == 0:
        z = x_abs ** y_abs
    else:
        z = _expnn(x_abs, y_abs, m_abs)
    neg = z != 0 and x_neg and y_abs != 0 and (y_abs & 1) == 1
    if neg and m_abs != 0:
        z = m_abs - z
        neg = False
    return -z if neg else z


def _expnn(x: int, y: int, m: int) -> int:
    """nat.expNN special cases (go:src/math/big/nat.go), m > 0."""
    if m == 1:
        return 0
    if y == 0:
        return 1
    if x == 0:
        return 0
    if x == 1:
        return 1
    if y == 1:
        return x % m
    return pow(x, y, m)


# ----------------------------------------------------------------- Paillier
# up:crypto/paillier/paillier.go (tss-lib v2.0.2), restated in SURVEY.md 8(a).

class ErrMessageTooLong(ValueError):
    pass


class ErrMessageMalFormed(ValueError):
    pass


def paillier_encrypt(N: int, m: int, r: int) -> int:
    """PublicKey.EncryptAndReturnRandomness with caller-supplied randomness r:
    c = Gamma^m * r^N mod N^2, Gamma = N+1.  Range check 0 <= m < N."""
    if m < 0 or m >= N:
        raise ErrMessageTooLong("message too long")
    N2 = N * N
    return (pow(N + 1, m, N2) * pow(r, N, N2)) % N2


def paillier_homo_mult(N: int, m: int, c1: int) -> int:
    """PublicKey.HomoMult: c1^m mod N^2 with 0 <= m < N and 0 <= c1 < N^2."""
    N2 = N * N
    if m < 0 or m >= N:
        raise ErrMessageTooLong("message too long")
    if c1 < 0 or c1 >= N2:
        raise ErrMessageTooLong("message too long")
    return pow(c1, m, N2)


def paillier_homo_add(N: int, c1: int, c2: int) -> int:
    """PublicKey.HomoAdd: c1*c2 mod N^2 with both in [0, N^2)."""
    N2 = N * N
    if c1 < 0 or c1 >= N2 or c2 < 0 or c2 >= N2:
        raise ErrMessageTooLong("message too long")
    return (c1 * c2) % N2


def paillier_L(u: int, N: int) -> int:
    """L(u) = (u - 1) / N."""
    return (u - 1) // N


def paillier_decrypt(N: int, lam: int, c: int) -> int:
    """PrivateKey.Decrypt: check range and gcd(c, N^2) == 1, then
    m = L(c^lambda mod N^2) * L(Gamma^lambda mod N^2)^-1 mod N."""
    N2 = N * N
    if c < 0 or c >= N2:
        raise ErrMessageTooLong("message too long")
    if math.gcd(c, N2) != 1:
        raise ErrMessageMalFormed("malformed message")
    lc = paillier_L(pow(c, lam, N2), N)
    lg = paillier_L(pow(N + 1, lam, N2), N)
    inv = mod_inverse(lg, N)
    return (lc * inv) % N


def paillier_lambda(p: int, q: int) -> int:
    """PrivateKey.LambdaN = lcm(p-1, q-1)."""
    phi = (p - 1) * (q - 1)
    return phi // math.gcd(p - 1, q - 1)


# ------------------------------------------------------------------ DRBG
class CounterDRBG:
    """Deterministic byte stream: SHA-256(b"mpcx-drbg" || seed_le64 || ctr_le64).

    The build's synthetic-input generator (not a tss-lib component): every
    fixture and bench input derives from it so C++/Go/Python can reproduce it.
    """

    def __init__(self, seed: int):
        self.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.ctr = 0
        self.buf = b""

    def read(self, n: int) -> bytes:
        while len(self.buf) < n:
            blk = hashlib.sha256(b"mpcx-drbg" + self.seed.to_bytes(8, "little") + self.ctr.to_bytes(8, "little")).digest()
            self.ctr += 1
            self.buf += blk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def randbelow(self, n: int) -> int:
        """Uniform in [0, n) by rejection on ceil(bits/8) bytes (top bits masked)."""
        if n <= 0:
            raise ValueError("n must be > 0")
        bits = n.bit_length()
        nbytes = (bits + 7) // 8
        mask = (1 << bits) - 1
        while True:
            v = int.from_bytes(self.read(nbytes), "big") & mask
            if v < n:
                return v

    def randbits(self, bits: int) -> int:
        nbytes = (bits + 7) // 8
        v = int.from_bytes(self.read(nbytes), "big")
        return v & ((1 << bits) - 1)

    def rand_coprime(self, n: int) -> int:
        """common.GetRandomPositiveRelativelyPrimeInt(n): uniform r in [1, n) with gcd(r, n) == 1."""
        while True:
            r = self.randbelow(n)
            if r > 0 and math.gcd(r, n) == 1:
                return r
