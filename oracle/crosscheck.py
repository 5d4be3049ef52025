"""ORACLE -- TEST INFRASTRUCTURE ONLY (see gomath.py header for the import rule).

Independent bignum implementations used to pin the oracle: GMP ``mpz_powm``
and OpenSSL ``BN_mod_exp`` via ctypes, plus the C restatement of Go's
expNNMontgomery (oracle/libgomodexp.so).  Each binding returns None if its
library is not loadable, so callers can report what was cross-checked.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))


class _Mpz(ctypes.Structure):
    _fields_ = [("alloc", ctypes.c_int), ("size", ctypes.c_int), ("d", ctypes.c_void_p)]


def _load(cands):
    for c in cands:
        try:
            return ctypes.CDLL(c)
        except OSError:
            continue
    return None


_gmp = _load(["/opt/conda/lib/libgmp.so.10", "libgmp.so.10", ctypes.util.find_library("gmp") or "libgmp.so"])
_ssl = _load(["libcrypto.so.3", "/usr/lib/x86_64-linux-gnu/libcrypto.so.3", ctypes.util.find_library("crypto") or "libcrypto.so"])


def gmp_powm(x: int, y: int, m: int) -> Optional[int]:
    if _gmp is None or y < 0 or m <= 0 or x < 0:
        return None
    init = _gmp.__gmpz_init
    set_str = _gmp.__gmpz_set_str
    powm = _gmp.__gmpz_powm
    get_str = _gmp.__gmpz_get_str
    get_str.restype = ctypes.c_void_p
    clear = _gmp.__gmpz_clear
    zs = [_Mpz() for _ in range(4)]
    for z in zs:
        init(ctypes.byref(z))
    try:
        set_str(ctypes.byref(zs[0]), ("%x" % x).encode(), 16)
        set_str(ctypes.byref(zs[1]), ("%x" % y).encode(), 16)
        set_str(ctypes.byref(zs[2]), ("%x" % m).encode(), 16)
        powm(ctypes.byref(zs[3]), ctypes.byref(zs[0]), ctypes.byref(zs[1]), ctypes.byref(zs[2]))
        p = get_str(None, 16, ctypes.byref(zs[3]))
        s = ctypes.string_at(p).decode()
        libc = ctypes.CDLL(None)
        libc.free(ctypes.c_void_p(p))
        return int(s, 16)
    finally:
        for z in zs:
            clear(ctypes.byref(z))


def openssl_mod_exp(x: int, y: int, m: int) -> Optional[int]:
    if _ssl is None or y < 0 or m <= 0 or x < 0:
        return None
    _ssl.BN_new.restype = ctypes.c_void_p
    _ssl.BN_CTX_new.restype = ctypes.c_void_p
    _ssl.BN_bn2hex.restype = ctypes.c_void_p
    _ssl.BN_bn2hex.argtypes = [ctypes.c_void_p]
    _ssl.BN_hex2bn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p]
    _ssl.BN_mod_exp.argtypes = [ctypes.c_void_p] * 5
    _ssl.BN_free.argtypes = [ctypes.c_void_p]
    _ssl.BN_CTX_free.argtypes = [ctypes.c_void_p]
    _ssl.CRYPTO_free.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
    bns = [ctypes.c_void_p(_ssl.BN_new()) for _ in range(4)]
    ctx = _ssl.BN_CTX_new()
    try:
        for b, v in zip(bns[:3], (x, y, m)):
            _ssl.BN_hex2bn(ctypes.byref(b), ("%x" % v).encode())
        if _ssl.BN_mod_exp(bns[3], bns[0], bns[1], bns[2], ctx) != 1:
            return None
        p = _ssl.BN_bn2hex(bns[3])
        s = ctypes.string_at(p).decode()
        _ssl.CRYPTO_free(p, b"crosscheck", 0)
        return int(s, 16) if s not in ("", "0") else 0
    finally:
        for b in bns:
            _ssl.BN_free(b)
        _ssl.BN_CTX_free(ctx)


def _words(v: int, n: int):
    return (ctypes.c_uint32 * n)(*[(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)])


def _from_words(arr, n: int) -> int:
    return sum(int(arr[i]) << (32 * i) for i in range(n))


_ARGS7 = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]


def load_c_oracle(word_bits: int = 32):
    """The C restatement of Go's expNN: word_bits 32 -> libgomodexp.so (the
    parity oracle), 64 -> libgomodexp64.so (Go's amd64 word size, the CPU
    baseline). Both expose gomodexp_expnn / gomodexp_montgomery over
    little-endian 32-bit words."""
    name = "libgomodexp.so" if word_bits == 32 else "libgomodexp64.so"
    path = os.path.join(_HERE, name)
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    if word_bits == 64:
        lib.gomodexp_expnn = lib.gomodexp64_expnn
        lib.gomodexp_montgomery = lib.gomodexp64_montgomery
    for f in ("gomodexp_expnn", "gomodexp_montgomery"):
        getattr(lib, f).argtypes = _ARGS7
        getattr(lib, f).restype = ctypes.c_int
    if word_bits == 32:
        lib.gomodexp_montgomery_batch.argtypes = _ARGS7
        lib.gomodexp_montgomery_batch.restype = ctypes.c_int
    return lib


class GmpPowm:
    """Repeated mpz_powm(x, y, m) on pre-set operands (CPU-baseline timing of
    GMP, a faster proxy for Go math/big); None-safe: .ok is False without
    libgmp."""

    def __init__(self, x: int, y: int, m: int):
        self.ok = _gmp is not None
        if not self.ok:
            return
        self.zs = [_Mpz() for _ in range(4)]
        g = lambda name: getattr(_gmp, name)  # noqa: E731 (no class-private name mangling)
        for z in self.zs:
            g("__gmpz_init")(ctypes.byref(z))
        for z, v in zip(self.zs, (x, y, m)):
            g("__gmpz_set_str")(ctypes.byref(z), ("%x" % v).encode(), 16)
        self._powm = g("__gmpz_powm")
        self._clear = g("__gmpz_clear")
        self._args = [ctypes.byref(self.zs[3]), ctypes.byref(self.zs[0]), ctypes.byref(self.zs[1]),
                      ctypes.byref(self.zs[2])]

    def run(self):
        self._powm(*self._args)

    def close(self):
        if self.ok:
            for z in self.zs:
                self._clear(ctypes.byref(z))
            self.ok = False


def gmp_version() -> Optional[str]:
    if _gmp is None:
        return None
    try:
        return ctypes.c_char_p.in_dll(_gmp, "__gmp_version").value.decode()
    except (ValueError, AttributeError):
        return "unknown"


def c_expnn(lib, x: int, y: int, m: int) -> Optional[int]:
    """x^y mod m through the C restatement of Go expNN (x, y >= 0, m > 0)."""
    nm = max(1, (m.bit_length() + 31) // 32)
    nx = max(1, (x.bit_length() + 31) // 32)
    ny = max(1, (y.bit_length() + 31) // 32)
    out = (ctypes.c_uint32 * nm)()
    rc = lib.gomodexp_expnn(out, _words(x, nx), nx, _words(y, ny), ny, _words(m, nm), nm)
    if rc != 0:
        return None
    return _from_words(out, nm)
