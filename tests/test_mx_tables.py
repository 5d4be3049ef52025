"""k_modexp_mx on the CPU: its constant tables (mpcx_mx_tables, host-only) against a
Python restatement, and the digit-level arithmetic of montmul_mx
(mpcium_amd/csrc/mpcx_mx.hpp) restated step by step in integers, so the bounds the
kernel relies on are checked on edge operands as well as random ones:
  - q (balanced radix-2^28 digits after ONE carry step) is a Montgomery quotient,
    |q| <= R/2 (1 + 2^-10), and every radix-2^7 byte of it is a valid signed i8;
  - every i8 column sum fits i32;
  - the carry out of the low half, rounded from its top four column sums, is exact;
  - U + m (the kernel's result) lies in (0, 2m) and is A B R^-1 mod m.
"""
import random

import pytest

from mpcium_amd import mpcx

DB = 28
M28 = (1 << 28) - 1
# MxShape (mpcx_internal.h) of the two MX geometries: L -> (D, table stride)
SHAPES = {148: (640, 720), 74: (352, 432)}


def digits(v, n, bits):
    return [(v >> (bits * i)) & ((1 << bits) - 1) for i in range(n)]


def lds_table(v7, L):
    """16 row copies of the reversed digit string: copy_i[x] = v7[D - x + i]."""
    D, stride = SHAPES[L]
    out = bytearray(16 * stride)
    for i in range(16):
        for x in range(stride):
            idx = D - x + i
            if 0 <= idx < len(v7):
                out[i * stride + x] = v7[idx]
    return bytes(out)


def fragment(tab, j, lane, L):
    """The 16 bytes lane (i, h) reads for Toeplitz block j (mx_toeplitz)."""
    D, stride = SHAPES[L]
    i, h = lane & 15, lane >> 4
    off = i * stride + 16 * (D // 16 - j + h)
    return tab[off:off + 16]


def i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def split(c, add):
    lo_sum = c[0] + ((c[1] & 0x1FFFFF) << 7) + ((c[2] & 0x3FFF) << 14) + ((c[3] & 0x7F) << 21) + add
    assert -(1 << 31) <= lo_sum < (1 << 31)
    return lo_sum, (c[1] >> 21) + (c[2] >> 14) + (c[3] >> 7)


def spread_bytes(e):
    x = e & 0xFFFFFFFF
    for msk in (0xFFFFFF80, 0xFFFF8000, 0xFF800000):
        x = (x + (x & msk)) & 0xFFFFFFFF
    return [((x >> (8 * i)) & 0xFF) - (256 if (x >> (8 * i)) & 0x80 else 0) for i in range(4)]


def conv(a, b, lo, hi):
    out = []
    for P in range(lo, hi):
        k0, k1 = max(0, P - len(b) + 1), min(P, len(a) - 1)
        out.append(sum(a[k] * b[P - k] for k in range(k0, k1 + 1)))
    return out


def montmul_mx_model(a, b, m, L=148):
    N7 = 4 * L
    RBITS = DB * L
    R = 1 << RBITS
    m2 = (-pow(m, -1, R)) % R
    T = a * b
    tl, th = digits(T % R, L, DB), digits(T >> RBITS, L, DB)
    c1 = conv(digits(T % R, N7, 7), digits(m2, N7, 7), 0, N7)
    assert max(c1) < 1 << 31
    e, hprev = [], 0
    for d in range(L):
        lo_sum, hi_sum = split(c1[4 * d:4 * d + 4], 1 << 27)
        e.append((lo_sum & M28) - (1 << 27) + hprev)
        hprev = hi_sum + (lo_sum >> 28)
    q7 = [v for ed in e for v in spread_bytes(ed)]
    assert all(-128 <= v <= 127 for v in q7)
    q = sum(v << (7 * i) for i, v in enumerate(q7))
    assert q == sum(v << (28 * i) for i, v in enumerate(e))
    assert (T + q * m) % R == 0
    assert abs(q) <= (R >> 1) + (R >> 11)
    m7 = digits(m, N7, 7)
    c2 = conv(q7, m7, 0, 2 * N7)
    assert max(abs(v) for v in c2) < 1 << 31
    lo_sum, hi_sum = split(c2[N7 - 4:N7], tl[L - 1] + (1 << 27))
    carry = hi_sum + (lo_sum >> 28)
    low = sum(c2[P] << (7 * P) for P in range(N7)) + (T % R)
    assert low % R == 0 and carry == low // R
    md, u, cin = digits(m, L, DB), [], carry
    for d in range(L):
        lo_sum, hi_sum = split(c2[N7 + 4 * d:N7 + 4 + 4 * d], th[d] + md[d])
        hi = hi_sum + (lo_sum >> 28)
        u.append(i32(lo_sum + (hi_sum << 28)) + cin if d == L - 1 else (lo_sum & M28) + cin)
        cin = hi
    U = sum(v << (28 * i) for i, v in enumerate(u))
    assert U == (T + q * m) // R + m
    return U, R


@pytest.mark.parametrize("L", [148, 74])
def test_mx_tables_match_restatement(L):
    rng = random.Random(L)
    R = 1 << (DB * L)
    top = min(DB * L - 3, 4096)  # 4m < R; the 4096-bit class's widest modulus
    for bits in (top, top - 1, top - 1000):
        m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        m2 = (-pow(m, -1, R)) % R
        v2, v1 = digits(m2, 4 * L, 7), digits(m, 4 * L, 7)
        img = mpcx.mx_tables(m, L)
        stride = SHAPES[L][1]
        assert img == lds_table(v2, L) + lds_table(v1, L)
        # each lane's read is the Toeplitz row it stands for: byte e of lane (i, h)
        # in block j = v7[16 j + i - 16 h - e]
        nj1 = (4 * L + 15) // 16
        nj2 = (4 * L + 62) // 16 + 1
        for tab, v7, nj in ((img[:16 * stride], v2, nj1), (img[16 * stride:], v1, nj2)):
            for j in (0, 1, nj // 2, nj - 1):
                for lane in (0, 5, 17, 33, 63):
                    i, h = lane & 15, lane >> 4
                    want = bytes(v7[16 * j + i - 16 * h - e] if 0 <= 16 * j + i - 16 * h - e < 4 * L else 0
                                 for e in range(16))
                    assert fragment(tab, j, lane, L) == want


def test_mx_tables_reject_bad_moduli():
    with pytest.raises(mpcx.MpcxError):
        mpcx.mx_tables(1 << 4000)  # even
    with pytest.raises(mpcx.MpcxError):
        mpcx.mx_tables((1 << 2071) - 1, 74)  # 4m >= R = 2^2072
    with pytest.raises(mpcx.MpcxError):
        mpcx.mx_tables(65537, 75)  # not an MX geometry


@pytest.mark.parametrize("L", [148, 74])
def test_mx_reduction_arithmetic(L):
    rng = random.Random(77 + L)
    top = min(DB * L - 3, 4096)
    cases = []
    for t in range(12):
        bits = (top, top, top - 1000, top // 2)[t % 4]
        m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if t == 1:
            m = (1 << top) - 1  # all-ones digits: the largest column sums
        cases += [(rng.randrange(2 * m), rng.randrange(2 * m), m), (2 * m - 1, 2 * m - 1, m), (0, 0, m), (1, 1, m)]
    for a, b, m in cases:
        U, R = montmul_mx_model(a, b, m, L)
        assert 0 < U < 2 * m
        assert U % m == a * b * pow(R, -1, m) % m


def test_mx_reduction_arithmetic_structured_moduli():
    # the moduli of tests/test_gpu_mx.py::test_mx_structured_moduli, with edge operands
    rng = random.Random(79)
    for m in ((1 << 4096) - 1, (1 << 4095) + 1, (1 << 4096) - (1 << 2048) - 1):
        for a, b in ((2 * m - 1, 2 * m - 1), (m - 1, m - 1), (1, 2 * m - 1), (0, 5),
                     (rng.randrange(2 * m), rng.randrange(2 * m))):
            U, R = montmul_mx_model(a, b, m, 148)
            assert 0 < U < 2 * m
            assert U % m == a * b * pow(R, -1, m) % m
