"""ctypes binding of the batched keygen / reshare proofs in libmpcx_host.so
(include/mpcx_host.h "keygen proofs"; C++ in csrc/host/proofs.cpp): tss-lib
v2.0.2 up:crypto/dlnproof, up:crypto/modproof, up:crypto/facproof with a batch
dimension (many proofs over the same public parameters). Every
exponentiation runs on the GPU through libmpcx.so. Proofs are dicts keyed by
the Go field names."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import host as _host
from .mpcx import ints_to_words, words_to_ints

W = 160  # integer width in 32-bit words (FacProof's v reaches ~4.9 kbit)
DLN_ITERATIONS, MOD_ITERATIONS = 128, 80
FAC_FIELDS = ["P", "Q", "A", "B", "T", "Sigma", "Z1", "Z2", "W1", "W2", "V"]

_vp, _u32, _u64, _i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int

SIGNATURES = [
    ("mpcxh_dln_prove_batch", _i, [_u32, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_dln_verify_batch", _i, [_u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_mod_prove_batch", _i, [_u32, _vp, _u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mpcxh_mod_verify_batch", _i, [_u32, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mpcxh_fac_prove_batch", _i, [_u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_fac_verify_batch", _i, [_u32, _vp, _u32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_bench_keygen_proofs", _i, [_u32, _vp, _u32, _u32, _u64, _u32, _vp, _vp]),
    ("mpcxh_bench_keygen_reshare", _i, [_u32, _vp, _u32, _u32, _u64, _u32, _i, ctypes.c_int64, _vp, _vp]),
]
_bound = False


def lib():
    global _bound
    l = _host.lib()
    if not _bound:
        for name, res, args in SIGNATURES:
            if not hasattr(l, name):  # an older build in an A/B run: its missing entries stay unbound
                continue
            f = getattr(l, name)
            f.restype, f.argtypes = res, args
        _bound = True
    return l


def _one(v: int) -> np.ndarray:
    return np.ascontiguousarray(ints_to_words([v], W)[0])


def _col(vals: Sequence[int]) -> np.ndarray:
    return np.ascontiguousarray(ints_to_words(list(vals), W))


def _sessions(ss: Sequence[bytes]):
    n = len(ss[0]) if ss else 0
    if any(len(s) != n for s in ss):
        raise ValueError("session ids must have equal length")
    return np.frombuffer(b"".join(ss), dtype=np.uint8).copy(), n


def _rows(a: np.ndarray, count: int, per: int) -> List[List[int]]:
    v = words_to_ints(a.reshape(count * per, W))
    return [v[i * per:(i + 1) * per] for i in range(count)]


def dln_prove(h1: int, h2: int, x: int, p: int, q: int, N: int, seeds: Sequence[int]) -> List[dict]:
    """NewDLNProof for len(seeds) proofs -> [{"Alpha": [...], "T": [...]}]."""
    n = len(seeds)
    args = [_one(v) for v in (h1, h2, x, p, q, N)]
    S = _host.Readers(seeds)
    al = np.zeros((n, DLN_ITERATIONS * W), dtype="<u4")
    t = np.zeros_like(al)
    _host._check(lib().mpcxh_dln_prove_batch(W, *[a.ctypes.data for a in args], n, S.ptr, al.ctypes.data,
                                             t.ctypes.data))
    return [{"Alpha": a, "T": b} for a, b in zip(_rows(al, n, DLN_ITERATIONS), _rows(t, n, DLN_ITERATIONS))]


def dln_verify(h1: int, h2: int, N: int, pfs: Sequence[dict]) -> List[bool]:
    n = len(pfs)
    args = [_one(v) for v in (h1, h2, N)]
    al = _col([v for p in pfs for v in p["Alpha"]])
    t = _col([v for p in pfs for v in p["T"]])
    ok = np.zeros(n, dtype=np.uint8)
    _host._check(lib().mpcxh_dln_verify_batch(W, *[a.ctypes.data for a in args], n, al.ctypes.data, t.ctypes.data,
                                              ok.ctypes.data))
    return [bool(x) for x in ok]


def mod_prove(sessions: Sequence[bytes], N: int, P: int, Q: int, seeds: Sequence[int]) -> List[dict]:
    n = len(seeds)
    ss, sl = _sessions(sessions)
    args = [_one(v) for v in (N, P, Q)]
    S = _host.Readers(seeds)
    Wv, A, B = (np.zeros((n, W), dtype="<u4") for _ in range(3))
    X, Z = (np.zeros((n, MOD_ITERATIONS * W), dtype="<u4") for _ in range(2))
    _host._check(lib().mpcxh_mod_prove_batch(W, ss.ctypes.data, sl, *[a.ctypes.data for a in args], n, S.ptr,
                                             Wv.ctypes.data, X.ctypes.data, A.ctypes.data, B.ctypes.data,
                                             Z.ctypes.data))
    return [{"W": w, "X": x, "A": a, "B": b, "Z": z} for w, x, a, b, z in
            zip(words_to_ints(Wv), _rows(X, n, MOD_ITERATIONS), words_to_ints(A), words_to_ints(B),
                _rows(Z, n, MOD_ITERATIONS))]


def mod_verify(sessions: Sequence[bytes], N: int, pfs: Sequence[dict]) -> List[bool]:
    n = len(pfs)
    ss, sl = _sessions(sessions)
    Nw = _one(N)
    Wv, A, B = _col([p["W"] for p in pfs]), _col([p["A"] for p in pfs]), _col([p["B"] for p in pfs])
    X = _col([v for p in pfs for v in p["X"]])
    Z = _col([v for p in pfs for v in p["Z"]])
    ok = np.zeros(n, dtype=np.uint8)
    _host._check(lib().mpcxh_mod_verify_batch(W, ss.ctypes.data, sl, Nw.ctypes.data, n, Wv.ctypes.data, X.ctypes.data,
                                              A.ctypes.data, B.ctypes.data, Z.ctypes.data, ok.ctypes.data))
    return [bool(x) for x in ok]


def fac_prove(sessions: Sequence[bytes], N0: int, NCap: int, s: int, t: int, N0p: int, N0q: int,
              seeds: Sequence[int]) -> List[dict]:
    n = len(seeds)
    ss, sl = _sessions(sessions)
    args = [_one(v) for v in (N0, NCap, s, t, N0p, N0q)]
    S = _host.Readers(seeds)
    pf = np.zeros((n, len(FAC_FIELDS) * W), dtype="<u4")
    neg = np.zeros(n, dtype=np.uint8)
    _host._check(lib().mpcxh_fac_prove_batch(W, ss.ctypes.data, sl, *[a.ctypes.data for a in args], n, S.ptr,
                                             pf.ctypes.data, neg.ctypes.data))
    out = []
    for row, ng in zip(_rows(pf, n, len(FAC_FIELDS)), neg):
        d = dict(zip(FAC_FIELDS, row))
        if ng:
            d["V"] = -d["V"]
        out.append(d)
    return out


def fac_verify(sessions: Sequence[bytes], N0: int, NCap: int, s: int, t: int, pfs: Sequence[dict]) -> List[bool]:
    """A proof with a field wider than the batch's W words (a peer's Sigma or V
    has no length bound on the wire) cannot cross the C-ABI: it is rejected here,
    as tss-lib rejects it (every field enters the challenge hash), and the rest
    of the batch is verified."""
    n = len(pfs)
    ss, sl = _sessions(sessions)
    args = [_one(v) for v in (N0, NCap, s, t)]
    lim = 1 << (32 * W)
    wide = [any(abs(p[f]) >= lim for f in FAC_FIELDS) for p in pfs]
    zero = dict.fromkeys(FAC_FIELDS, 0)
    pfs = [zero if w else p for p, w in zip(pfs, wide)]  # all-zero fields fail the range checks
    pf = _col([abs(p[f]) for p in pfs for f in FAC_FIELDS])
    neg = np.array([1 if p["V"] < 0 else 0 for p in pfs], dtype=np.uint8)
    ok = np.zeros(n, dtype=np.uint8)
    _host._check(lib().mpcxh_fac_verify_batch(W, ss.ctypes.data, sl, *[a.ctypes.data for a in args], n,
                                              pf.ctypes.data, neg.ctypes.data, ok.ctypes.data))
    return [bool(x) and not w for x, w in zip(ok, wide)]


class _Party(ctypes.Structure):
    _fields_ = [("N", _vp), ("LambdaN", _vp), ("P", _vp), ("Q", _vp), ("NTilde", _vp), ("h1", _vp), ("h2", _vp),
                ("alpha", _vp), ("beta", _vp), ("p", _vp), ("q", _vp)]


KEYGEN_STATS = ["prove_s", "verify_s", "total_s", "sessions", "parties", "proofs", "verifications", "failures",
                "engine_busy_s", "alg_macs", "waves", "wave_sessions", "max_wave_s"]
RESHARE_STATS = KEYGEN_STATS + ["keygen_sessions", "reshare_sessions", "keygen_wave_s", "reshare_wave_s",
                                "vss_checks", "vss_failures"]


def bench_keygen_proofs(parties: Sequence[dict], sessions: int, seed: int = 0x6B67, wave: int = 0,
                        trace: bool = False, reshare: bool = False, tamper_session: int = -1):
    """Config-5 driver (csrc/host/keygenload.hpp): the DLN / Mod / Fac proof
    work of `sessions` keygen sessions of len(parties) nodes, streamed in waves
    of `wave` sessions (0: the driver's default, 1024), two waves in flight;
    reshare=True: every odd wave is a resharing wave (the new committee's proof
    work plus the old committee's VSS and its checks, mpcium's two resharing
    sessions per node), so a keygen and a reshare wave are in flight together.
    parties: dicts with N, LambdaN, P, Q, NTildei, H1i, H2i, Alpha, Beta, p, q.
    trace: also return one traced session per wave -- [{"session": s,
    "digests": {(i, "dln1"|"dln2"|"mod"): d, (i, "fac", j): d}, "verified":
    count} + for reshare waves "vss": {"old": [d_i], "new_shares": d,
    "passed": count}]."""
    keep = []

    def ptr(v):
        a = _one(v)
        keep.append(a)
        return a.ctypes.data

    arr = (_Party * len(parties))()
    for k, n in enumerate(parties):
        arr[k] = _Party(ptr(n["N"]), ptr(n["LambdaN"]), ptr(n["P"]), ptr(n["Q"]), ptr(n["NTildei"]), ptr(n["H1i"]),
                        ptr(n["H2i"]), ptr(n["Alpha"]), ptr(n["Beta"]), ptr(n["p"]), ptr(n["q"]))
    names = RESHARE_STATS if reshare else KEYGEN_STATS
    st = np.zeros(len(names), dtype=np.float64)
    n = len(parties)
    wv = wave or 1024
    n_waves = (sessions + wv - 1) // wv
    tk = 1 + n * (3 + (n - 1)) * 8 + 1
    tw = tk + (n * 8 + 9 if reshare else 0)
    tr = np.zeros(max(1, n_waves * tw), dtype="<u4")
    if reshare:
        rc = lib().mpcxh_bench_keygen_reshare(W, arr, n, sessions, seed, wave, 1, tamper_session, st.ctypes.data,
                                              tr.ctypes.data if trace else None)
    else:
        rc = lib().mpcxh_bench_keygen_proofs(W, arr, n, sessions, seed, wave, st.ctypes.data,
                                             tr.ctypes.data if trace else None)
    _host._check(rc)
    stats = dict(zip(names, [float(x) for x in st]))
    if not trace:
        return stats
    out = []
    for w in range(n_waves):
        o = tr[w * tw:(w + 1) * tw]
        d, k = {}, 1
        for i in range(n):
            for kind in ("dln1", "dln2", "mod"):
                d[(i, kind)] = words_to_ints(o[k:k + 8].reshape(1, 8))[0]
                k += 8
            for j in range(n):
                if j != i:
                    d[(i, "fac", j)] = words_to_ints(o[k:k + 8].reshape(1, 8))[0]
                    k += 8
        t = {"session": int(o[0]), "digests": d, "verified": int(o[k])}
        if reshare and w % 2 == 1:
            v = o[tk:]
            t["vss"] = {"old": [words_to_ints(v[8 * i:8 * i + 8].reshape(1, 8))[0] for i in range(n)],
                        "new_shares": words_to_ints(v[8 * n:8 * n + 8].reshape(1, 8))[0],
                        "passed": int(v[8 * n + 8])}
        out.append(t)
    return stats, out
