"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (mpcium_amd/) never imports it.

Pure-Python restatement of the tss-lib v2.0.2 helpers the MtA sub-protocol
uses (module pinned at /root/reference/go.mod:10, source absent from the image;
"up:" = github.com/bnb-chain/tss-lib/v2).  Every function names the upstream
function it restates; details marked "upstream, verify" are restated from the
published algorithm and could not be checked against the source here
(no Go toolchain, tss-lib not vendored).

* Randomness: Go crypto/rand.Int(reader, max) (go:src/crypto/rand/util.go) over
  a caller-supplied io.Reader; common.MustGetRandomInt, GetRandomPositiveInt,
  GetRandomPositiveRelativelyPrimeInt, IsNumberInMultiplicativeGroup
  (up:common/random.go).
* Hashing: common.SHA512_256, SHA512_256i, SHA512_256i_TAGGED
  (up:common/hash.go; 8-byte little-endian element-count prefix, then per
  element its big.Int.Bytes(), a '$' delimiter and its byte length as 8
  little-endian bytes -- restated from tss-lib v2's hash.go as recalled, no
  source in this image to check it against: upstream, verify) and
  common.RejectionSample (up:common/hash_utils.go: eHash mod q -- upstream,
  verify).
* secp256k1 (tss.EC() = btcec/v2 S256, /root/reference/go.mod:29): affine
  double-and-add; ScalarBaseMult(k) = (k mod n)*G, the semantics under which
  MtAwc's u = alpha*G / s1*G == e*X + u check holds (alpha < q^3).
"""
from __future__ import annotations

import hashlib
import math
import struct
from typing import Optional, Sequence, Tuple

# ------------------------------------------------------------ io.Reader
class Reader:
    """Per-session io.Reader stand-in: the build's CounterDRBG byte stream
    (SHA-256(b"mpcx-drbg" || seed_le64 || ctr_le64)), identical to
    oracle/gomath.py CounterDRBG and the C++ host's CounterDRBG."""

    def __init__(self, seed: int):
        self.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.ctr = 0
        self.buf = b""

    def read(self, n: int) -> bytes:
        while len(self.buf) < n:
            self.buf += hashlib.sha256(b"mpcx-drbg" + self.seed.to_bytes(8, "little")
                                       + self.ctr.to_bytes(8, "little")).digest()
            self.ctr += 1
        out, self.buf = self.buf[:n], self.buf[n:]
        return out


def crypto_rand_int(rd: Reader, mx: int) -> int:
    """go crypto/rand.Int(rand, max): uniform in [0, max) by rejection on
    k = ceil(bitlen(max-1)/8) big-endian bytes with the top byte masked to
    bitlen(max-1) % 8 bits."""
    if mx <= 0:
        raise ValueError("crypto/rand: argument to Int is <= 0")
    n = mx - 1
    bit_len = n.bit_length()
    if bit_len == 0:
        return 0
    k = (bit_len + 7) // 8
    b = bit_len % 8
    if b == 0:
        b = 8
    while True:
        bz = bytearray(rd.read(k))
        bz[0] &= (1 << b) - 1
        v = int.from_bytes(bz, "big")
        if v < mx:
            return v


def must_get_random_int(rd: Reader, bits: int) -> int:
    """common.MustGetRandomInt(rand, bits): crypto/rand.Int(rand, 2^bits - 1)."""
    if bits <= 0 or bits > 5000:
        raise ValueError("MustGetRandomInt: bits should be positive, non-zero and less than 5000")
    return crypto_rand_int(rd, (1 << bits) - 1)


def get_random_positive_int(rd: Reader, less_than: int) -> Optional[int]:
    """common.GetRandomPositiveInt(rand, lessThan): MustGetRandomInt(bitlen)
    until < lessThan."""
    if less_than is None or less_than <= 0:
        return None
    while True:
        t = must_get_random_int(rd, less_than.bit_length())
        if t < less_than:
            return t


def is_number_in_multiplicative_group(n: int, v: int) -> bool:
    """common.IsNumberInMultiplicativeGroup(n, v): 1 <= v < n and gcd(v, n) == 1."""
    return 1 <= v < n and math.gcd(v, n) == 1


def get_random_positive_relatively_prime_int(rd: Reader, n: int) -> Optional[int]:
    """common.GetRandomPositiveRelativelyPrimeInt(rand, n)."""
    if n is None or n <= 0:
        return None
    while True:
        t = must_get_random_int(rd, n.bit_length())
        if is_number_in_multiplicative_group(n, t):
            return t


def is_in_interval(b: int, bound: int) -> bool:
    """common.IsInInterval(b, bound): 0 <= b < bound (upstream, verify)."""
    return 0 <= b < bound


# ------------------------------------------------------------ hashing
HASH_INPUT_DELIMITER = b"$"


def _bytes(n: Optional[int]) -> bytes:
    """big.Int.Bytes(): minimal big-endian magnitude, b"" for 0 (nil -> zero)."""
    if not n:
        return b""
    return abs(n).to_bytes((abs(n).bit_length() + 7) // 8, "big")


def _frame(parts: Sequence[bytes]) -> bytes:
    """8-byte little-endian part count, then per part: its bytes, '$', and its
    length as 8 little-endian bytes (the audit's domain separation: the capacity
    len(inLenBz) + bzSize + inLen + inLen*8 of up:common/hash.go)."""
    data = struct.pack("<Q", len(parts))
    for p in parts:
        data += p + HASH_INPUT_DELIMITER + struct.pack("<Q", len(p))
    return data


def sha512_256(*parts: bytes) -> Optional[bytes]:
    """common.SHA512_256(in ...[]byte)."""
    if not parts:
        return None
    return hashlib.new("sha512_256", _frame(parts)).digest()


def sha512_256i(*ints: int) -> Optional[int]:
    """common.SHA512_256i(in ...*big.Int)."""
    if not ints:
        return None
    return int.from_bytes(hashlib.new("sha512_256", _frame([_bytes(x) for x in ints])).digest(), "big")


def sha512_256i_tagged(tag: bytes, *ints: int) -> Optional[int]:
    """common.SHA512_256i_TAGGED(tag, in ...*big.Int): SHA512/256 over
    SHA512_256(tag) || SHA512_256(tag) || framed inputs."""
    tag_bz = sha512_256(tag)
    if not ints:
        return None
    h = hashlib.new("sha512_256")
    h.update(tag_bz)
    h.update(tag_bz)
    h.update(_frame([_bytes(x) for x in ints]))
    return int.from_bytes(h.digest(), "big")


def rejection_sample(q: int, e_hash: int) -> int:
    """common.RejectionSample(q, eHash) = eHash mod q (upstream, verify)."""
    return e_hash % q


# ------------------------------------------------------------ secp256k1
SECP_P = 2 ** 256 - 2 ** 32 - 977
SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
SECP_G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
          0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)

Point = Optional[Tuple[int, int]]  # None = point at infinity


def ec_on_curve(P: Point) -> bool:
    if P is None:
        return False
    x, y = P
    return 0 <= x < SECP_P and 0 <= y < SECP_P and (y * y - x * x * x - 7) % SECP_P == 0


def ec_add(P: Point, Q: Point) -> Point:
    if P is None:
        return Q
    if Q is None:
        return P
    (x1, y1), (x2, y2) = P, Q
    if x1 == x2:
        if (y1 + y2) % SECP_P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, SECP_P) % SECP_P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, SECP_P) % SECP_P
    x3 = (lam * lam - x1 - x2) % SECP_P
    return x3, (lam * (x1 - x3) - y1) % SECP_P


def ec_mul(k: int, P: Point) -> Point:
    """k*P with k reduced mod n (the group order)."""
    k %= SECP_N
    R: Point = None
    while k:
        if k & 1:
            R = ec_add(R, P)
        P = ec_add(P, P)
        k >>= 1
    return R


def scalar_base_mult(k: int) -> Point:
    """crypto.ScalarBaseMult(ec, k) = (k mod n) * G."""
    return ec_mul(k, SECP_G)
