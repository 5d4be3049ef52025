"""ctypes binding of libmpcx.so (include/mpcx.h).

Integers cross the boundary as little-endian 32-bit words, operand-major.
No fallback: if libmpcx.so is missing or the GPU call fails, an exception is
raised.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libmpcx.so")

MPCX_OK, MPCX_EINVAL, MPCX_ENODEV, MPCX_EHIP, MPCX_ENOMEM = 0, 1, 2, 3, 4

_u32p = ctypes.POINTER(ctypes.c_uint32)
_vp = ctypes.c_void_p

# (name, restype, argtypes) -- must match include/mpcx.h
SIGNATURES = [
    ("mpcx_version", ctypes.c_int, []),
    ("mpcx_set_option", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    ("mpcx_get_option", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    ("mpcx_last_error", ctypes.c_char_p, []),
    ("mpcx_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("mpcx_init", ctypes.c_int, [ctypes.c_int]),
    ("mpcx_init_devices", ctypes.c_int, [ctypes.c_int]),
    ("mpcx_bound_devices", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("mpcx_select_device", ctypes.c_int, [ctypes.c_int]),
    ("mpcx_device_launches", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    ("mpcx_kernel_stats", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]),
    ("mpcx_partition", ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, _u32p, _u32p, _u32p]),
    ("mpcx_shutdown", ctypes.c_int, []),
    ("mpcx_modulus_register", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    ("mpcx_modulus_release", ctypes.c_int, [_vp]),
    ("mpcx_modulus_info", ctypes.c_int, [_vp, _u32p, _u32p]),
    ("mpcx_modulus_geometry", ctypes.c_int, [_vp, _u32p, _u32p, _u32p, _u32p]),
    ("mpcx_mx_tables", ctypes.c_int, [_u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    ("mpcx_modexp_batch", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                         ctypes.c_int, _vp, ctypes.c_uint32]),
    ("mpcx_modexp_batch_device", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                                ctypes.c_int, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    ("mpcx_modexp_mul_batch", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                             ctypes.c_int, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32]),
    ("mpcx_modexp_mul_batch_device", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp,
                                                    ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, _vp,
                                                    ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    ("mpcx_modexp_submit", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                          ctypes.c_int, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                          ctypes.POINTER(_vp)]),
    ("mpcx_job_test", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    ("mpcx_job_wait", ctypes.c_int, [_vp]),
    ("mpcx_mulmod_batch", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp,
                                         ctypes.c_uint32]),
    ("mpcx_fermat2_batch", ctypes.c_int, [ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    ("mpcx_ec_combine_batch", ctypes.c_int, [ctypes.c_uint32, _vp, _vp, _vp]),
    ("mpcx_modexp_multi_batch", ctypes.c_int, [ctypes.c_uint32, _vp]),
    ("mpcx_mr_batch", ctypes.c_int, [ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp]),
    ("mpcx_fixedbase_register", ctypes.c_int, [_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    ("mpcx_fixedbase_release", ctypes.c_int, [_vp]),
    ("mpcx_fixedbase_info", ctypes.c_int, [_vp, _u32p, ctypes.POINTER(ctypes.c_size_t)]),
    ("mpcx_fixedbase_exp_batch", ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(_vp), ctypes.c_uint32,
                                                ctypes.POINTER(_vp), _u32p, _vp, ctypes.c_uint32, _vp,
                                                ctypes.c_uint32]),
    ("mpcx_fixedbase_multi_batch", ctypes.c_int, [ctypes.c_uint32, _vp]),
    ("mpcx_lucas_batch", ctypes.c_int, [ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp]),
    ("mpcx_safeprime_step", ctypes.c_int, [ctypes.c_uint64, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           _vp, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p, _vp, _vp, _vp]),
    ("mpcx_safeprime_sieve_fermat", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u32p,
                                                   _vp, _vp]),
    ("mpcx_dev_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_vp)]),
    ("mpcx_dev_free", ctypes.c_int, [_vp]),
    ("mpcx_host_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("mpcx_host_free", ctypes.c_int, [_vp]),
    ("mpcx_copy_stats", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    ("mpcx_memcpy_h2d", ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    ("mpcx_memcpy_d2h", ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    ("mpcx_stream_create", ctypes.c_int, [ctypes.POINTER(_vp)]),
    ("mpcx_stream_destroy", ctypes.c_int, [_vp]),
    ("mpcx_stream_sync", ctypes.c_int, [_vp]),
    ("mpcx_sync", ctypes.c_int, [_vp]),
]


class MpcxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mpcx error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """Load libmpcx.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # MPCX_LIB_PATH: another build of libmpcx.so (an earlier round's, for
        # interleaved A/B timing of the same bench command); symbols it lacks
        # stay unbound
        path = os.environ.get("MPCX_LIB_PATH") or _LIB_PATH
        if not os.path.exists(path):
            raise MpcxError(MPCX_ENODEV, f"{path} not built: run `python -m mpcium_amd.build`")
        l = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            if path != _LIB_PATH and not hasattr(l, name):
                continue
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _check(rc: int):
    if rc != MPCX_OK:
        raise MpcxError(rc, lib().mpcx_last_error().decode(errors="replace"))


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().mpcx_device_count(ctypes.byref(n)))
    return n.value


def init(device: int = 0):
    _check(lib().mpcx_init(device))


def init_devices(n_gpus: int = 0):
    """Bind GPUs 0..n_gpus-1 (0: all visible) in this process."""
    _check(lib().mpcx_init_devices(n_gpus))


def bound_devices() -> List[int]:
    n = ctypes.c_int(0)
    ords = (ctypes.c_int * 16)()
    _check(lib().mpcx_bound_devices(ctypes.byref(n), ords, 16))
    return list(ords[:n.value])


def partition(count: int, n_devices: int, min_slice: int = 4096):
    """[(first, n)] slice plan of a host-buffer batch over n_devices GPUs."""
    f = (ctypes.c_uint32 * 16)()
    n = (ctypes.c_uint32 * 16)()
    k = ctypes.c_uint32(0)
    _check(lib().mpcx_partition(count, n_devices, min_slice, f, n, ctypes.byref(k)))
    return [(f[i], n[i]) for i in range(k.value)]


def device_launches(index: int) -> int:
    v = ctypes.c_uint64(0)
    _check(lib().mpcx_device_launches(index, ctypes.byref(v)))
    return v.value


def kernel_stats(reset: bool = False) -> dict:
    """mpcx_kernel_stats: per-kernel launches, operands, Go-equivalent MACs and
    GPU ms since the last reset (collected while set_option("kernel_stats", 1))."""
    import json
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mpcx_kernel_stats(buf, len(buf), 1 if reset else 0))
    return json.loads(buf.value.decode())


def copy_stats() -> dict:
    """mpcx_copy_stats: host bytes DMA'd directly from/to mpcx_host_alloc
    blocks, bytes bounced through the lanes' pinned buffers, bounce allocations."""
    v = [ctypes.c_uint64(0) for _ in range(3)]
    _check(lib().mpcx_copy_stats(*(ctypes.byref(x) for x in v)))
    return {"direct_bytes": v[0].value, "bounced_bytes": v[1].value, "bounce_allocs": v[2].value}


MX_TABLE_BYTES = {148: 2 * 16 * 720, 74: 2 * 16 * 432}


def mx_tables(m: int, L: int = 148) -> bytes:
    """mpcx_mx_tables: the LDS image of k_modexp_mx's Toeplitz tables of
    m'' = -m^-1 mod 2^(28 L) and of m (host-only, no device needed)."""
    w = int_to_words(m, 128)
    n = MX_TABLE_BYTES.get(L, 0)
    out = ctypes.create_string_buffer(max(n, 1))
    _check(lib().mpcx_mx_tables(w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 128, L, out, n))
    return out.raw


def select_device(index: int):
    _check(lib().mpcx_select_device(index))


def set_option(key: str, value: int):
    _check(lib().mpcx_set_option(key.encode(), int(value)))


def get_option(key: str) -> int:
    v = ctypes.c_int(0)
    _check(lib().mpcx_get_option(key.encode(), ctypes.byref(v)))
    return v.value


def shutdown():
    _check(lib().mpcx_shutdown())


# ----------------------------------------------------------- int <-> words
def int_to_words(v: int, n: int) -> np.ndarray:
    if v < 0:
        raise ValueError("negative integers do not cross the C-ABI")
    return np.frombuffer(v.to_bytes(4 * n, "little"), dtype="<u4").copy()


def ints_to_words(vals: Sequence[int], n: int) -> np.ndarray:
    buf = b"".join(int(v).to_bytes(4 * n, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), n).copy()


def words_to_ints(arr: np.ndarray) -> List[int]:
    arr = np.ascontiguousarray(arr, dtype="<u4")
    n = arr.shape[1]
    raw = arr.tobytes()
    return [int.from_bytes(raw[i * 4 * n:(i + 1) * 4 * n], "little") for i in range(arr.shape[0])]


def nwords(v: int) -> int:
    return max(1, (v.bit_length() + 31) // 32)


class Modulus:
    """A registered odd modulus (mpcx_modulus_register)."""

    def __init__(self, m: int):
        if m <= 0:
            raise ValueError("modulus must be positive")
        self.m = m
        w = int_to_words(m, nwords(m))
        h = _vp()
        _check(lib().mpcx_modulus_register(w.ctypes.data, len(w), ctypes.byref(h)))
        self._h = h
        bits, cw = ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().mpcx_modulus_info(h, ctypes.byref(bits), ctypes.byref(cw)))
        self.bits, self.class_words = bits.value, cw.value
        g = [ctypes.c_uint32() for _ in range(4)]
        _check(lib().mpcx_modulus_geometry(h, *[ctypes.byref(x) for x in g]))
        self.L, self.P, self.K, self.G = (x.value for x in g)
        self.words = nwords(m)

    @property
    def handle(self):
        return self._h

    def release(self):
        if self._h:
            _check(lib().mpcx_modulus_release(self._h))
            self._h = None

    def exp_words(self, bases: np.ndarray, exps: np.ndarray, shared: bool, out_words: Optional[int] = None) -> np.ndarray:
        """Raw word-level batch: bases (count, bw) uint32, exps (ew,) or (count, ew)."""
        bases = np.ascontiguousarray(bases, dtype="<u4")
        exps = np.ascontiguousarray(exps, dtype="<u4")
        count, bw = bases.shape
        ew = exps.shape[-1] if exps.size else 0
        ow = out_words or self.words
        out = np.zeros((count, ow), dtype="<u4")
        _check(lib().mpcx_modexp_batch(self._h, count, bases.ctypes.data, bw,
                                       exps.ctypes.data if exps.size else None, ew, 1 if shared else 0,
                                       out.ctypes.data, ow))
        return out

    def _operands(self, vals: Sequence[int], what: str) -> np.ndarray:
        bw = self.class_words
        lim = 1 << (32 * bw)
        if any(v < 0 or v >= lim for v in vals):
            raise ValueError(f"{what} must be in [0, 2^(32*class_words)); reduce mod m first")
        return ints_to_words(vals, bw)

    def mulmod(self, a: Sequence[int], b: Sequence[int]) -> List[int]:
        """[a_i * b_i mod m] (mpcx_mulmod_batch)."""
        if len(a) != len(b):
            raise ValueError("length mismatch")
        if len(a) == 0:
            return []
        A, B = self._operands(a, "a"), self._operands(b, "b")
        out = np.zeros((len(a), self.words), dtype="<u4")
        _check(lib().mpcx_mulmod_batch(self._h, len(a), A.ctypes.data, A.shape[1], B.ctypes.data, B.shape[1],
                                       out.ctypes.data, self.words))
        return words_to_ints(out)

    def exp_mul(self, bases: Sequence[int], exps: Union[int, Sequence[int]], muls: Sequence[int]) -> List[int]:
        """[mul_i * b_i^e_i mod m] (mpcx_modexp_mul_batch)."""
        if len(muls) != len(bases):
            raise ValueError("one multiplier per base")
        if len(bases) == 0:
            return []
        B = self._operands(bases, "bases")
        Mu = self._operands(muls, "muls")
        E, shared = self._exps(exps, len(bases))
        out = np.zeros((len(bases), self.words), dtype="<u4")
        _check(lib().mpcx_modexp_mul_batch(self._h, len(bases), B.ctypes.data, B.shape[1],
                                           E.ctypes.data if E.size else None, E.shape[-1] if E.size else 0,
                                           1 if shared else 0, Mu.ctypes.data, Mu.shape[1], out.ctypes.data,
                                           self.words))
        return words_to_ints(out)

    @staticmethod
    def _exps(exps, count):
        if isinstance(exps, int):
            if exps < 0:
                raise ValueError("negative exponent")
            return (int_to_words(exps, nwords(exps)) if exps else np.zeros(0, dtype="<u4")), True
        if len(exps) != count:
            raise ValueError("one exponent per base")
        if any(e < 0 for e in exps):
            raise ValueError("negative exponent")
        ew = max(nwords(e) for e in exps)
        return ints_to_words(exps, ew), False

    def submit(self, bases: Sequence[int], exps: Union[int, Sequence[int]]) -> "Job":
        """Asynchronous [b^e mod m] (mpcx_modexp_submit); Job.wait() -> list."""
        B = self._operands(bases, "bases")
        E, shared = self._exps(exps, len(bases))
        out = np.zeros((len(bases), self.words), dtype="<u4")
        h = _vp()
        _check(lib().mpcx_modexp_submit(self._h, len(bases), B.ctypes.data, B.shape[1],
                                        E.ctypes.data if E.size else None, E.shape[-1] if E.size else 0,
                                        1 if shared else 0, None, 0, out.ctypes.data, self.words, ctypes.byref(h)))
        return Job(h, (B, E, out), lambda: words_to_ints(out))

    def exp(self, bases: Sequence[int], exps: Union[int, Sequence[int]]) -> List[int]:
        """[b^e mod m] for non-negative ints; `exps` is one shared int or one per base."""
        if len(bases) == 0:
            return []
        B = self._operands(bases, "bases")
        E, shared = self._exps(exps, len(bases))
        return words_to_ints(self.exp_words(B, E, shared))


class ModexpGroup(ctypes.Structure):
    """mpcx_modexp_group_t"""
    _fields_ = [("mod", _vp), ("count", ctypes.c_uint32), ("bases", _vp), ("base_words", ctypes.c_uint32),
                ("exps", _vp), ("exp_words", ctypes.c_uint32), ("exp_shared", ctypes.c_int), ("muls", _vp),
                ("mul_words", ctypes.c_uint32), ("out", _vp), ("out_words", ctypes.c_uint32)]


def modexp_multi(groups) -> List[List[int]]:
    """Several batches in one launch (mpcx_modexp_multi_batch): groups of
    (Modulus, bases, exps: one shared int or one per base, muls or None) ->
    [[mul_i * b_i^e_i mod m] per group]."""
    keep, outs = [], []
    arr = (ModexpGroup * max(1, len(groups)))()
    for i, (mod, bases, exps, muls) in enumerate(groups):
        B = mod._operands(bases, "bases")
        E, shared = Modulus._exps(exps, len(bases))
        Mu = mod._operands(muls, "muls") if muls is not None else None
        out = np.zeros((len(bases), mod.words), dtype="<u4")
        keep += [B, E, Mu]
        outs.append(out)
        arr[i] = ModexpGroup(mod.handle, len(bases), B.ctypes.data if len(bases) else None, mod.class_words,
                             E.ctypes.data if E.size else None, E.shape[-1] if E.size else 0, 1 if shared else 0,
                             Mu.ctypes.data if Mu is not None else None, mod.class_words if Mu is not None else 0,
                             out.ctypes.data if len(bases) else None, mod.words)
    _check(lib().mpcx_modexp_multi_batch(len(groups), arr))
    return [words_to_ints(o) if o.shape[0] else [] for o in outs]


class Job:
    """An mpcx_job_t: keeps the submitted buffers alive until wait()."""

    def __init__(self, h, bufs, result):
        self._h, self._bufs, self._result = h, bufs, result

    def done(self) -> bool:
        d = ctypes.c_int(0)
        _check(lib().mpcx_job_test(self._h, ctypes.byref(d)))
        return bool(d.value)

    def wait(self):
        h, self._h = self._h, None
        if h is None:
            raise RuntimeError("job already waited")
        _check(lib().mpcx_job_wait(h))
        r = self._result()
        self._bufs = None
        return r


class FixedBase:
    """A comb table for a long-lived base of a registered modulus of <= 2080
    bits (mpcx_fixedbase_register): exponents of up to `max_exp_bits` bits."""

    def __init__(self, mod: Modulus, base: int, max_exp_bits: int):
        self.mod, self.base = mod, base % mod.m
        w = mod._operands([self.base], "base")
        h = _vp()
        _check(lib().mpcx_fixedbase_register(mod.handle, w.ctypes.data, w.shape[1], max_exp_bits, ctypes.byref(h)))
        self._h = h
        mb, tb = ctypes.c_uint32(), ctypes.c_size_t()
        _check(lib().mpcx_fixedbase_info(h, ctypes.byref(mb), ctypes.byref(tb)))
        self.max_exp_bits, self.table_bytes = mb.value, tb.value

    @property
    def handle(self):
        return self._h

    def release(self):
        if self._h:
            _check(lib().mpcx_fixedbase_release(self._h))
            self._h = None


def fixedbase_exp(fbs: Sequence[FixedBase], exps: Sequence[Sequence[int]],
                  muls: Optional[Sequence[int]] = None) -> List[int]:
    """[mul_i * prod_t b_t^(e_t,i) mod m] (mpcx_fixedbase_exp_batch); exps[t][i]."""
    nb = len(fbs)
    if nb != len(exps) or nb == 0:
        raise ValueError("one exponent list per fixed base")
    count = len(exps[0])
    if any(len(e) != count for e in exps):
        raise ValueError("exponent lists differ in length")
    if count == 0:
        return []
    mod = fbs[0].mod
    Es = []
    for e in exps:
        if any(v < 0 for v in e):
            raise ValueError("negative exponent")
        ew = max(nwords(v) for v in e)
        Es.append(ints_to_words(e, ew))
    Mu = mod._operands(muls, "muls") if muls is not None else None
    out = np.zeros((count, mod.words), dtype="<u4")
    hs = (_vp * nb)(*[f.handle for f in fbs])
    eps = (_vp * nb)(*[E.ctypes.data for E in Es])
    ews = (ctypes.c_uint32 * nb)(*[E.shape[1] for E in Es])
    _check(lib().mpcx_fixedbase_exp_batch(nb, hs, count, eps, ews, Mu.ctypes.data if Mu is not None else None,
                                          Mu.shape[1] if Mu is not None else 0, out.ctypes.data, mod.words))
    return words_to_ints(out)


class FixedBaseGroup(ctypes.Structure):
    """mpcx_fixedbase_group_t"""
    _fields_ = [("nbases", ctypes.c_uint32), ("fbs", _vp * 2), ("count", ctypes.c_uint32), ("exps", _vp * 2),
                ("exp_words", ctypes.c_uint32 * 2), ("muls", _vp), ("mul_words", ctypes.c_uint32), ("out", _vp),
                ("out_words", ctypes.c_uint32)]


def fixedbase_multi(groups) -> List[List[int]]:
    """Several comb batches in one launch (mpcx_fixedbase_multi_batch): groups
    of (fixed bases, exps[t][i], muls or None) -> [[mul_i * prod_t b_t^e_t,i mod m]
    per group]; the groups' moduli share one size class."""
    keep, outs = [], []
    arr = (FixedBaseGroup * max(1, len(groups)))()
    for i, (fbs, exps, muls) in enumerate(groups):
        nb = len(fbs)
        if nb != len(exps) or not 1 <= nb <= 2:
            raise ValueError("one exponent list per fixed base (1 or 2)")
        count = len(exps[0])
        mod = fbs[0].mod
        g = FixedBaseGroup()
        g.nbases, g.count = nb, count
        for t in range(nb):
            E = ints_to_words(exps[t], max([nwords(v) for v in exps[t]] + [1]))
            keep.append(E)
            g.fbs[t] = fbs[t].handle
            g.exps[t] = E.ctypes.data if count else None
            g.exp_words[t] = E.shape[1]
        Mu = mod._operands(muls, "muls") if muls is not None else None
        keep.append(Mu)
        g.muls = Mu.ctypes.data if Mu is not None else None
        g.mul_words = mod.class_words if Mu is not None else 0
        out = np.zeros((count, mod.words), dtype="<u4")
        outs.append(out)
        g.out = out.ctypes.data if count else None
        g.out_words = mod.words
        arr[i] = g
    _check(lib().mpcx_fixedbase_multi_batch(len(groups), arr))
    return [words_to_ints(o) if o.shape[0] else [] for o in outs]


def exp_batch(m: int, bases: Sequence[int], exps: Union[int, Sequence[int]]) -> List[int]:
    mod = Modulus(m)
    try:
        return mod.exp(bases, exps)
    finally:
        mod.release()


SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141  # secp256k1 group order


def ec_combine_batch(items) -> list:
    """secp256k1 a G + b P + c Q per item (a, b, c, P, Q), points as (x, y)
    tuples or None (infinity) -> list of (x, y) or None. Scalars are any
    integers, taken mod the group order n (as the C++ CombineBatch does)."""
    n = len(items)
    if n == 0:
        return []
    sc = np.zeros((n, 24), dtype="<u4")
    pt = np.zeros((n, 32), dtype="<u4")
    mask = (1 << 256) - 1
    for i, (a, b, c, P, Q) in enumerate(items):
        a, b, c = a % SECP_N, b % SECP_N, c % SECP_N
        sc[i] = int_to_words(a | (b << 256) | (c << 512), 24)
        px = (P[0] | (P[1] << 256)) if P is not None else 0
        qx = (Q[0] | (Q[1] << 256)) if Q is not None else 0
        pt[i] = int_to_words(px | (qx << 512), 32)
    out = np.zeros((n, 16), dtype="<u4")
    _check(lib().mpcx_ec_combine_batch(n, sc.ctypes.data, pt.ctypes.data, out.ctypes.data))
    res = []
    for v in words_to_ints(out):
        res.append(None if v == 0 else (v & mask, v >> 256))
    return res


def fermat2_batch(cands: Sequence[int]) -> List[bool]:
    """[2^(p-1) mod p == 1] for odd candidates p (5 <= p < 2^1024)."""
    if len(cands) == 0:
        return []
    pw = max(nwords(p) for p in cands)
    P = ints_to_words(cands, pw)
    ok = np.zeros(len(cands), dtype=np.uint8)
    _check(lib().mpcx_fermat2_batch(len(cands), P.ctypes.data, pw, ok.ctypes.data))
    return [bool(x) for x in ok]


def mr_batch(ns: Sequence[int], bases: Sequence[int]) -> List[bool]:
    """[n is a strong probable prime to base a] for odd n (5 <= n < 2^1024)."""
    if len(ns) != len(bases):
        raise ValueError("one base per candidate")
    if len(ns) == 0:
        return []
    w = max(nwords(n) for n in ns)
    Nw = ints_to_words(ns, w)
    A = ints_to_words([b % n if b.bit_length() > 32 * w else b for b, n in zip(bases, ns)], w)
    ok = np.zeros(len(ns), dtype=np.uint8)
    _check(lib().mpcx_mr_batch(len(ns), Nw.ctypes.data, w, A.ctypes.data, ok.ctypes.data))
    return [bool(x) for x in ok]


def lucas_batch(ns: Sequence[int], Ps: Sequence[int]) -> List[bool]:
    """[n passes the strong Lucas test with parameter P] (mpcx_lucas_batch)."""
    if len(ns) != len(Ps):
        raise ValueError("one P per candidate")
    if len(ns) == 0:
        return []
    w = max(nwords(n) for n in ns)
    Nw = ints_to_words(ns, w)
    Pw = np.array(Ps, dtype="<u4")
    ok = np.zeros(len(ns), dtype=np.uint8)
    _check(lib().mpcx_lucas_batch(len(ns), Nw.ctypes.data, w, Pw.ctypes.data, ok.ctypes.data))
    return [bool(x) for x in ok]


def safeprime_step(seed: int, stream_off: int, count: int, q_bits: int, sprp_q: Sequence[int] = (),
                   raw: Optional[bytes] = None, max_pass: int = 4096):
    """mpcx_safeprime_step: (n_sieved, [(index in the step, p)] Fermat passes,
    [strong-test verdicts of sprp_q]); candidates from stream byte stream_off."""
    W = 32
    Q = ints_to_words(list(sprp_q), W) if len(sprp_q) else np.zeros((0, W), dtype="<u4")
    pidx = np.zeros(max(max_pass, 1), dtype=np.uint32)
    pp = np.zeros((max(max_pass, 1), W), dtype="<u4")
    sok = np.zeros(max(len(sprp_q), 1), dtype=np.uint8)
    ns, npass = ctypes.c_uint32(), ctypes.c_uint32()
    rb = None
    if raw is not None:
        rb = np.frombuffer(raw, dtype=np.uint8).copy()
    _check(lib().mpcx_safeprime_step(seed, rb.ctypes.data if rb is not None else None, stream_off, count, q_bits,
                                     Q.ctypes.data if len(sprp_q) else None, len(sprp_q), max_pass,
                                     ctypes.byref(ns), ctypes.byref(npass), pidx.ctypes.data, pp.ctypes.data,
                                     sok.ctypes.data))
    k = npass.value
    return ns.value, list(zip((int(i) for i in pidx[:k]), words_to_ints(pp[:k]))), [bool(x) for x in sok[:len(sprp_q)]]


def safeprime_sieve_fermat(raw: bytes, q_bits: int):
    """GPU candidate batch (mpcx_safeprime_sieve_fermat): [(index, fermat_ok)]
    for the sieve survivors among len(raw) // nbytes candidates."""
    nb = (q_bits + 7) // 8
    count = len(raw) // nb
    buf = np.frombuffer(raw[:count * nb], dtype=np.uint8).copy()
    idx = np.zeros(max(count, 1), dtype="<u4")
    ok = np.zeros(max(count, 1), dtype=np.uint8)
    n = ctypes.c_uint32()
    _check(lib().mpcx_safeprime_sieve_fermat(buf.ctypes.data, nb, count, q_bits, ctypes.byref(n), idx.ctypes.data,
                                             ok.ctypes.data))
    return [(int(i), bool(o)) for i, o in zip(idx[:n.value], ok[:n.value])]
