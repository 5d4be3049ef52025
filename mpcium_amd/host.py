"""ctypes binding of libmpcx_host.so (include/mpcx_host.h): the C++ mirror of
tss-lib's ModInt.Exp, crypto/paillier and safe-prime / preparams generation.
Same names and error behaviour as the Go API, with a batch dimension."""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .mpcx import MpcxError, ints_to_words, nwords, words_to_ints

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libmpcx_host.so")
_vp, _u32, _u64, _i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int

RAND_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t)


class ReaderT(ctypes.Structure):
    """mpcxh_reader_t: one session's io.Reader (fn, ctx) or CounterDRBG seed."""
    _fields_ = [("fn", _vp), ("ctx", _vp), ("seed", _u64)]


class Readers:
    """A ctypes array of mpcxh_reader_t for a batch. Each source is an int
    (the CounterDRBG seed) or an object with .read(n) -> bytes (an io.Reader,
    called back from libmpcx_host's worker threads). Keep the object alive
    for the duration of the call."""

    def __init__(self, sources):
        self._cbs = []
        arr = (ReaderT * max(1, len(sources)))()
        for i, s in enumerate(sources):
            if isinstance(s, (int, np.integer)):
                arr[i].seed = int(s) & 0xFFFFFFFFFFFFFFFF
            else:
                def read(_ctx, buf, n, _s=s):
                    b = _s.read(n)
                    if len(b) != n:
                        raise ValueError("short read")
                    ctypes.memmove(buf, b, n)
                cb = RAND_FN(read)
                self._cbs.append(cb)
                arr[i].fn = ctypes.cast(cb, _vp)
        self.arr = arr

    @property
    def ptr(self):
        return ctypes.addressof(self.arr)

SIGNATURES = [
    ("mpcxh_last_error", ctypes.c_char_p, []),
    ("mpcxh_init", _i, [_i]),
    ("mpcxh_init_devices", _i, [_i]),
    ("mpcxh_modint_exp_batch", _i, [_vp, _u32, _u32, _vp, _u32, _vp, _vp, _u32, _vp, _i, _vp, _u32, _vp]),
    ("mpcxh_paillier_encrypt_batch", _i, [_vp, _u32, _u32, _vp, _u32, _vp, _vp, _u32, _vp, _u32, _vp]),
    ("mpcxh_paillier_homomult_batch", _i, [_vp, _u32, _u32, _vp, _u32, _vp, _vp, _u32, _vp, _vp, _u32, _vp]),
    ("mpcxh_paillier_homoadd_batch", _i, [_vp, _u32, _u32, _vp, _u32, _vp, _vp, _u32, _vp, _vp, _u32, _vp]),
    ("mpcxh_paillier_decrypt_batch", _i, [_vp, _u32, _vp, _u32, _vp, _u32, _vp, _u32, _u32, _vp, _u32, _vp, _vp,
                                          _u32, _vp]),
    ("mpcxh_safe_primes", _i, [_i, _i, _u64, _vp, _vp, _vp, _vp, _u32, _vp, _vp]),
    ("mpcxh_safe_prime_batch", _i, [_i, _u64, _u64, _u32, _u32, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_generate_preparams", _i, [_u64, _vp, _vp, _vp, _vp]),
    ("mpcxh_candidate_from_bytes", _i, [_vp, ctypes.c_size_t, _i, _vp, _u32]),
    ("mpcxh_probably_prime_batch", _i, [_u32, _vp, _u32, _i, _vp]),
    ("mpcxh_coprime_batch", _i, [_u32, _vp, _vp, _u32, _vp]),
    ("mpcxh_profile_report", _i, [ctypes.c_char_p, ctypes.c_size_t, _i]),
    ("mpcxh_host_threads", _i, [_vp, _vp]),
    ("mpcxh_pinned_pool_stats", _i, [_vp, _vp, _vp, _vp]),
    ("mpcxh_pool_selftest", _i, [_u32, _u32, _u32, _vp]),
    ("mpcxh_nat_arith", _i, [_i, _vp, _u32, _vp, _u32, _vp, _u32, _vp]),
    ("mpcxh_drbg_read", _i, [_u64, _vp, ctypes.c_size_t]),
    ("mpcxh_go_rand_int63", _i, [ctypes.c_int64, _u32, _vp]),
    ("mpcxh_go_mr_bases", _i, [_vp, _u32, _u32, _vp]),
]

ERR_OK, ERR_MESSAGE_TOO_LONG, ERR_MESSAGE_MALFORMED = 0, 1, 2
STAT_KEYS = ["candidates", "sieved_out", "fermat_tests", "mr_tests", "usec", "lucas_tests"]
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise MpcxError(2, f"{_LIB_PATH} not built: run `python -m mpcium_amd.build`")
        l = ctypes.CDLL(_LIB_PATH)
        for name, res, args in SIGNATURES:
            if not hasattr(l, name):  # an older build in an A/B run: its missing entries stay unbound
                continue
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _check(rc):
    if rc != 0:
        raise MpcxError(rc, lib().mpcxh_last_error().decode(errors="replace"))


def init(device: int = 0):
    _check(lib().mpcxh_init(device))


def init_devices(n_gpus: int = 0):
    """Bind GPUs 0..n_gpus-1 (0: every visible GPU) in this process."""
    _check(lib().mpcxh_init_devices(n_gpus))


def _signed(vals: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
    w = max([nwords(abs(v)) for v in vals] + [1])
    return ints_to_words([abs(v) for v in vals], w), np.array([1 if v < 0 else 0 for v in vals], dtype=np.uint8)


def _w(v: int) -> np.ndarray:
    return ints_to_words([v], nwords(v))[0]


def modint_exp(m: int, xs: Sequence[int], ys, shared: Optional[bool] = None) -> List[Optional[int]]:
    """Go common.ModInt(m).Exp semantics; None where Go returns nil."""
    if isinstance(ys, int):
        ys, shared = [ys], True
    shared = bool(shared) if shared is not None else len(ys) == 1 and len(xs) != 1
    X, xn = _signed(xs)
    Y, yn = _signed(ys)
    M = _w(m)
    ow = len(M)
    out = np.zeros((len(xs), ow), dtype="<u4")
    ok = np.zeros(len(xs), dtype=np.uint8)
    _check(lib().mpcxh_modint_exp_batch(M.ctypes.data, len(M), len(xs), X.ctypes.data, X.shape[1], xn.ctypes.data,
                                        Y.ctypes.data, Y.shape[1], yn.ctypes.data, 1 if shared else 0,
                                        out.ctypes.data, ow, ok.ctypes.data))
    return [z if k else None for z, k in zip(words_to_ints(out), ok)]


class PublicKey:
    """crypto/paillier.PublicKey (batched)."""

    def __init__(self, N: int):
        self.N = N
        self._Nw = _w(N)

    def _out(self, n, words):
        return np.zeros((n, words), dtype="<u4"), np.zeros(n, dtype=np.uint8)

    def encrypt(self, ms: Sequence[int], rs: Sequence[int]):
        """EncryptAndReturnRandomness with supplied r: ([c or None], [err])."""
        Mw, mn = _signed(ms)
        R = ints_to_words(rs, max(nwords(r) for r in rs))
        cw = 2 * len(self._Nw)
        c, err = self._out(len(ms), cw)
        _check(lib().mpcxh_paillier_encrypt_batch(self._Nw.ctypes.data, len(self._Nw), len(ms), Mw.ctypes.data,
                                                  Mw.shape[1], mn.ctypes.data, R.ctypes.data, R.shape[1],
                                                  c.ctypes.data, cw, err.ctypes.data))
        return words_to_ints(c), [int(e) for e in err]

    def encrypt_words(self, Mw: np.ndarray, mn: np.ndarray, R: np.ndarray):
        """encrypt on little-endian word arrays (count x words; mn: 1 where m < 0):
        the same C-ABI call without the Python-int conversions -> (c words, err)."""
        cw = 2 * len(self._Nw)
        c, err = self._out(Mw.shape[0], cw)
        _check(lib().mpcxh_paillier_encrypt_batch(self._Nw.ctypes.data, len(self._Nw), Mw.shape[0], Mw.ctypes.data,
                                                  Mw.shape[1], mn.ctypes.data, R.ctypes.data, R.shape[1],
                                                  c.ctypes.data, cw, err.ctypes.data))
        return c, err

    def homo_mult_words(self, Mw: np.ndarray, mn: np.ndarray, C: np.ndarray, cn: np.ndarray):
        """homo_mult on word arrays (as encrypt_words) -> (words, err)."""
        ow = 2 * len(self._Nw)
        o, err = self._out(Mw.shape[0], ow)
        _check(lib().mpcxh_paillier_homomult_batch(self._Nw.ctypes.data, len(self._Nw), Mw.shape[0], Mw.ctypes.data,
                                                   Mw.shape[1], mn.ctypes.data, C.ctypes.data, C.shape[1],
                                                   cn.ctypes.data, o.ctypes.data, ow, err.ctypes.data))
        return o, err

    def homo_mult(self, ms: Sequence[int], c1s: Sequence[int]):
        Mw, mn = _signed(ms)
        C, cn = _signed(c1s)
        ow = 2 * len(self._Nw)
        o, err = self._out(len(ms), ow)
        _check(lib().mpcxh_paillier_homomult_batch(self._Nw.ctypes.data, len(self._Nw), len(ms), Mw.ctypes.data,
                                                   Mw.shape[1], mn.ctypes.data, C.ctypes.data, C.shape[1],
                                                   cn.ctypes.data, o.ctypes.data, ow, err.ctypes.data))
        return words_to_ints(o), [int(e) for e in err]

    def homo_add(self, c1s: Sequence[int], c2s: Sequence[int]):
        A, an = _signed(c1s)
        B, bn = _signed(c2s)
        ow = 2 * len(self._Nw)
        o, err = self._out(len(c1s), ow)
        _check(lib().mpcxh_paillier_homoadd_batch(self._Nw.ctypes.data, len(self._Nw), len(c1s), A.ctypes.data,
                                                  A.shape[1], an.ctypes.data, B.ctypes.data, B.shape[1],
                                                  bn.ctypes.data, o.ctypes.data, ow, err.ctypes.data))
        return words_to_ints(o), [int(e) for e in err]


class PrivateKey(PublicKey):
    def __init__(self, N: int, lambda_n: int, P: int, Q: int):
        super().__init__(N)
        self.LambdaN, self.P, self.Q = lambda_n, P, Q

    def decrypt(self, cs: Sequence[int]):
        C, cn = _signed(cs)
        lw, pw, qw = _w(self.LambdaN), _w(self.P), _w(self.Q)
        mw = len(self._Nw)
        m, err = self._out(len(cs), mw)
        _check(lib().mpcxh_paillier_decrypt_batch(self._Nw.ctypes.data, len(self._Nw), lw.ctypes.data, len(lw),
                                                  pw.ctypes.data, len(pw), qw.ctypes.data, len(qw), len(cs),
                                                  C.ctypes.data, C.shape[1], cn.ctypes.data, m.ctypes.data, mw,
                                                  err.ctypes.data))
        return words_to_ints(m), [int(e) for e in err]


def safe_primes(bit_len: int, num: int, seed: int = 0, rand_fn=None):
    """[(p, q, index)] in candidate-stream order + stats dict."""
    words = (bit_len + 31) // 32
    P = np.zeros((num, words), dtype="<u4")
    Q = np.zeros((num, words), dtype="<u4")
    idx = np.zeros(num, dtype=np.uint64)
    st = np.zeros(6, dtype=np.uint64)
    cb = RAND_FN(rand_fn) if rand_fn else None
    _check(lib().mpcxh_safe_primes(bit_len, num, seed, ctypes.cast(cb, _vp) if cb else None, None, P.ctypes.data,
                                   Q.ctypes.data, words, idx.ctypes.data, st.ctypes.data))
    stats = dict(zip(STAT_KEYS, (int(x) for x in st)))
    return list(zip(words_to_ints(P), words_to_ints(Q), (int(i) for i in idx))), stats


def safe_prime_batch(bit_len: int, seed: int, batch_no: int, batch: int = 0, max_out: int = 64):
    """One batch of the CounterDRBG(seed) candidate stream (sharded search):
    [(p, q, index)] of its accepted safe primes in stream order + stats dict."""
    words = (bit_len + 31) // 32
    P = np.zeros((max_out, words), dtype="<u4")
    Q = np.zeros((max_out, words), dtype="<u4")
    idx = np.zeros(max_out, dtype=np.uint64)
    st = np.zeros(6, dtype=np.uint64)
    n = ctypes.c_uint32(0)
    _check(lib().mpcxh_safe_prime_batch(bit_len, seed, batch_no, batch, max_out, P.ctypes.data, Q.ctypes.data, words,
                                        idx.ctypes.data, ctypes.byref(n), st.ctypes.data))
    k = n.value
    stats = dict(zip(STAT_KEYS, (int(x) for x in st)))
    return list(zip(words_to_ints(P[:k]), words_to_ints(Q[:k]), (int(i) for i in idx[:k]))), stats


PREPARAM_FIELDS = ["N", "LambdaN", "PhiN", "P", "Q", "NTildei", "H1i", "H2i", "Alpha", "Beta", "p", "q"]


def generate_preparams(seed: int = 0, rand_fn=None):
    out = np.zeros((len(PREPARAM_FIELDS), 64), dtype="<u4")
    st = np.zeros(6, dtype=np.uint64)
    cb = RAND_FN(rand_fn) if rand_fn else None
    _check(lib().mpcxh_generate_preparams(seed, ctypes.cast(cb, _vp) if cb else None, None, out.ctypes.data,
                                          st.ctypes.data))
    vals = dict(zip(PREPARAM_FIELDS, words_to_ints(out)))
    stats = dict(zip(STAT_KEYS, (int(x) for x in st)))
    return vals, stats


def host_threads() -> tuple:
    """(threads parallel loops use now, usable CPUs of this process)."""
    t, u = ctypes.c_int(0), ctypes.c_int(0)
    _check(lib().mpcxh_host_threads(ctypes.byref(t), ctypes.byref(u)))
    return t.value, u.value


def pool_selftest(tasks: int, outer: int, inner: int) -> int:
    s = ctypes.c_uint64(0)
    _check(lib().mpcxh_pool_selftest(tasks, outer, inner, ctypes.byref(s)))
    return s.value


def nat_arith(op: int, a: int, b: int) -> int:
    """Host bignum op (test hook): 0 a*b, 1 a//b, 2 a%b, 3 a^-1 mod b, 4 gcd."""
    def words(x):
        n = max(1, (x.bit_length() + 31) // 32)
        return (ctypes.c_uint32 * n)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]), (n if x else 0)
    wa, na = words(a)
    wb, nb = words(b)
    nout = na + nb + 2
    out, ow = (ctypes.c_uint32 * nout)(), ctypes.c_uint32(0)
    _check(lib().mpcxh_nat_arith(op, wa, na, wb, nb, out, nout, ctypes.byref(ow)))
    return sum(int(out[i]) << (32 * i) for i in range(ow.value))


def profile_report(reset: bool = False) -> str:
    """Host-time profile (MPCX_HOST_PROFILE=1), '' when off."""
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mpcxh_profile_report(buf, len(buf), 1 if reset else 0))
    return buf.value.decode()


def pinned_pool_stats() -> dict:
    """mpcxh_pinned_pool_stats: the engine's page-locked staging pool (bytes
    held, peak bytes in use) and the pageable fallbacks taken when pinning failed."""
    v = [ctypes.c_uint64(0) for _ in range(4)]
    _check(lib().mpcxh_pinned_pool_stats(*(ctypes.byref(x) for x in v)))
    return {"held_bytes": v[0].value, "peak_in_use_bytes": v[1].value, "fallbacks": v[2].value,
            "fallback_bytes": v[3].value}


def probably_prime(ns: Sequence[int], reps: int = 20) -> List[bool]:
    """Go (*Int).ProbablyPrime(reps) decisions (mpcxh_probably_prime_batch)."""
    if len(ns) == 0:
        return []
    w = max(nwords(n) for n in ns)
    Nw = ints_to_words(list(ns), w)
    ok = np.zeros(len(ns), dtype=np.uint8)
    _check(lib().mpcxh_probably_prime_batch(len(ns), Nw.ctypes.data, w, reps, ok.ctypes.data))
    return [bool(x) for x in ok]


def coprime(xs: Sequence[int], ms: Sequence[int]) -> List[bool]:
    """gcd(x, m) == 1 for odd m (mpcxh_coprime_batch, host side)."""
    if len(xs) != len(ms):
        raise ValueError("coprime: sizes")
    if len(xs) == 0:
        return []
    w = max(nwords(v) for v in list(xs) + list(ms))
    X, M = ints_to_words(list(xs), w), ints_to_words(list(ms), w)
    ok = np.zeros(len(xs), dtype=np.uint8)
    _check(lib().mpcxh_coprime_batch(len(xs), X.ctypes.data, M.ctypes.data, w, ok.ctypes.data))
    return [bool(v) for v in ok]


def candidate_from_bytes(raw: bytes, q_bit_len: int) -> int:
    words = (q_bit_len + 31) // 32 + 1
    out = np.zeros(words, dtype="<u4")
    buf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    _check(lib().mpcxh_candidate_from_bytes(buf, len(raw), q_bit_len, out.ctypes.data, words))
    return words_to_ints(out[None, :])[0]


def drbg_read(seed: int, n: int) -> bytes:
    buf = (ctypes.c_uint8 * n)()
    _check(lib().mpcxh_drbg_read(seed, buf, n))
    return bytes(buf)


def go_rand_int63(seed: int, count: int) -> list:
    """Go math/rand: the first `count` Int63() of rand.New(rand.NewSource(seed)) (test hook)."""
    out = np.zeros(count, dtype=np.int64)
    _check(lib().mpcxh_go_rand_int63(seed, count, out.ctypes.data))
    return [int(v) for v in out]


def go_mr_bases(n: int, reps: int) -> list:
    """The `reps` Miller-Rabin bases Go's ProbablyPrime(reps) draws for odd n > 3 (test hook)."""
    w = (n.bit_length() + 31) // 32
    src = ints_to_words([n], w)
    out = np.zeros((reps, w), dtype="<u4")
    _check(lib().mpcxh_go_mr_bases(src.ctypes.data, w, reps, out.ctypes.data))
    return words_to_ints(out)
