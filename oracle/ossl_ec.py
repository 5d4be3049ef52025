"""ORACLE -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline legs).

secp256k1 point arithmetic through OpenSSL's libcrypto (EC_POINT_mul /
EC_POINT_add over NID_secp256k1), a C-speed stand-in for btcec/v2
(/root/reference/go.mod:29) when the signing oracle (oracle/signing_ref.py,
oracle/mta_ref.py) is timed as the host-CPU baseline. install() swaps it into
oracle/tss_ref.py's ec_mul / ec_add / scalar_base_mult; the results are the
same points (checked against the pure-Python restatement in
tests/test_signing_cpu.py). Each process that calls install() owns one BN_CTX.
"""
from __future__ import annotations

import ctypes
import time

from . import tss_ref as T

NID_SECP256K1 = 714
_vp = ctypes.c_void_p


class _Ec:
    def __init__(self):
        L = ctypes.CDLL("libcrypto.so.3")
        for name, res, args in (
                ("EC_GROUP_new_by_curve_name", _vp, [ctypes.c_int]),
                ("EC_POINT_new", _vp, [_vp]), ("EC_POINT_free", None, [_vp]),
                ("EC_POINT_mul", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
                ("EC_POINT_add", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
                ("EC_POINT_is_at_infinity", ctypes.c_int, [_vp, _vp]),
                ("EC_POINT_set_affine_coordinates", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
                ("EC_POINT_get_affine_coordinates", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
                ("BN_CTX_new", _vp, []), ("BN_new", _vp, []), ("BN_free", None, [_vp]),
                ("BN_bin2bn", _vp, [ctypes.c_char_p, ctypes.c_int, _vp]),
                ("BN_bn2bin", ctypes.c_int, [_vp, ctypes.c_char_p]),
                ("BN_num_bits", ctypes.c_int, [_vp])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L
        self.g = L.EC_GROUP_new_by_curve_name(NID_SECP256K1)
        self.ctx = L.BN_CTX_new()
        self.bx, self.by, self.bk, self.bk2 = L.BN_new(), L.BN_new(), L.BN_new(), L.BN_new()
        self.p1, self.p2, self.r = L.EC_POINT_new(self.g), L.EC_POINT_new(self.g), L.EC_POINT_new(self.g)
        self.c_seconds = 0.0  # time inside libcrypto calls (CPU-baseline Python share)

    def _bn(self, v: int, bn):
        b = v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")
        self.L.BN_bin2bn(b, len(b), bn)
        return bn

    def _int(self, bn) -> int:
        n = (self.L.BN_num_bits(bn) + 7) // 8
        buf = ctypes.create_string_buffer(max(1, n))
        self.L.BN_bn2bin(bn, buf)
        return int.from_bytes(buf.raw[:n], "big")

    def _set(self, pt, P):
        self.L.EC_POINT_set_affine_coordinates(self.g, pt, self._bn(P[0], self.bx), self._bn(P[1], self.by), self.ctx)

    def _get(self, pt):
        if self.L.EC_POINT_is_at_infinity(self.g, pt):
            return None
        self.L.EC_POINT_get_affine_coordinates(self.g, pt, self.bx, self.by, self.ctx)
        return self._int(self.bx), self._int(self.by)

    def mul(self, k: int, P) -> T.Point:
        k %= T.SECP_N
        if P is None or k == 0:
            return None
        t0 = time.perf_counter()
        self._set(self.p1, P)
        self.L.EC_POINT_mul(self.g, self.r, None, self.p1, self._bn(k, self.bk), self.ctx)
        out = self._get(self.r)
        self.c_seconds += time.perf_counter() - t0
        return out

    def base(self, k: int) -> T.Point:
        k %= T.SECP_N
        if k == 0:
            return None
        t0 = time.perf_counter()
        self.L.EC_POINT_mul(self.g, self.r, self._bn(k, self.bk), None, None, self.ctx)
        out = self._get(self.r)
        self.c_seconds += time.perf_counter() - t0
        return out

    def add(self, P, Q) -> T.Point:
        if P is None:
            return Q
        if Q is None:
            return P
        t0 = time.perf_counter()
        self._set(self.p1, P)
        self._set(self.p2, Q)
        self.L.EC_POINT_add(self.g, self.r, self.p1, self.p2, self.ctx)
        out = self._get(self.r)
        self.c_seconds += time.perf_counter() - t0
        return out


_ec = None


def install() -> "_Ec":
    """Route tss_ref's ec_mul / ec_add / scalar_base_mult through OpenSSL."""
    global _ec
    if _ec is None:
        _ec = _Ec()
    T.ec_mul = _ec.mul
    T.ec_add = _ec.add
    T.scalar_base_mult = _ec.base
    return _ec
