"""ctypes binding of the batched MtA / MtAwc mirror in libmpcx_host.so
(include/mpcx_host.h "MtA"; C++ in csrc/host/mta.cpp): tss-lib v2.0.2
up:crypto/mta/{share_protocol,range_proof,proofs}.go with a batch dimension.

Same names, argument meaning and error behaviour as the Go functions
(AliceInit, BobMid, BobMidWC, AliceEnd, AliceEndWC, the proofs' Verify), for a
batch of sessions that share key material; every exponentiation runs on the
GPU through libmpcx.so. Integers are Python ints; proofs are dicts keyed by the
Go field names; points are (x, y) tuples.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import host as _host
from .mpcx import ints_to_words, words_to_ints

W = 128  # integer width in 32-bit words (N^2 of a 2048-bit Paillier key)
RANGE_FIELDS = ["Z", "U", "W", "S", "S1", "S2"]
BOB_FIELDS = ["Z", "ZPrm", "T", "V", "W", "S", "S1", "S2", "T1", "T2"]
ERR_OK, ERR_MESSAGE_TOO_LONG, ERR_MESSAGE_MALFORMED, ERR_PROOF_VERIFY = 0, 1, 2, 3

_vp, _u32, _u64, _i, _sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t


class PaillierKey(ctypes.Structure):
    _fields_ = [("N", _vp), ("LambdaN", _vp), ("P", _vp), ("Q", _vp)]


class DLN(ctypes.Structure):
    _fields_ = [("NTilde", _vp), ("h1", _vp), ("h2", _vp), ("P", _vp), ("Q", _vp)]


SIGNATURES = [
    ("mpcxh_mta_alice_init_batch", _i, [_u32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("mpcxh_mta_verify_range_alice_batch", _i, [_u32, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("mpcxh_mta_bob_mid_batch", _i, [_u32, _vp, _u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp]),
    ("mpcxh_mta_verify_bob_batch", _i, [_u32, _vp, _u32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("mpcxh_mta_alice_end_batch", _i, [_u32, _vp, _u32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mpcxh_mta_bob_mid_pair_batch", _i, [_u32, _vp, _u32, _vp, _vp, _vp, _u32] + [_vp] * 17),
    ("mpcxh_mta_alice_end_pair_batch", _i, [_u32, _vp, _u32, _vp, _vp, _u32] + [_vp] * 10),
    ("mpcxh_sha512_256i", _i, [_vp, _sz, _u32, _vp, _u32, _vp]),
    ("mpcxh_secp_scalar_base_mult", _i, [_vp, _u32, _vp]),
    ("mpcxh_secp_scalar_mult", _i, [_vp, _vp, _u32, _vp]),
    ("mpcxh_secp_lincomb", _i, [_vp, _vp, _vp, _u32, _vp]),
    ("mpcxh_random_draws", _i, [_u64, _vp, _u32, _i, _u32, _vp]),
    ("mpcxh_bench_signing", _i, [_u32, _vp, _vp, _u32, _u32, _u32, _u64, _vp, _u32, _vp, ctypes.c_int64, _i]),
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
            f.restype = res
            f.argtypes = args
        _bound = True
    return l


def _check(rc):
    _host._check(rc)


def _col(vals: Sequence[int]) -> np.ndarray:
    return np.ascontiguousarray(ints_to_words(list(vals), W))


def _one(v: Optional[int]) -> Optional[np.ndarray]:
    return None if v is None else np.ascontiguousarray(ints_to_words([v], W)[0])


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


class _Keep:
    """Holds the numpy buffers a ctypes struct points into."""

    def __init__(self):
        self.bufs = []

    def arr(self, v):
        a = _one(v)
        self.bufs.append(a)
        return _ptr(a)


def _paillier(keep: _Keep, N: int, LambdaN: Optional[int] = None, P: Optional[int] = None,
              Q: Optional[int] = None) -> PaillierKey:
    return PaillierKey(keep.arr(N), keep.arr(LambdaN), keep.arr(P), keep.arr(Q))


def _dln(keep: _Keep, d: Dict[str, int]) -> DLN:
    return DLN(keep.arr(d["NTilde"]), keep.arr(d["h1"]), keep.arr(d["h2"]), keep.arr(d.get("P")),
               keep.arr(d.get("Q")))


def _proofs(buf: np.ndarray, fields: List[str], count: int, wc: bool = False) -> List[dict]:
    vals = words_to_ints(buf.reshape(count * buf.shape[1] // W, W))
    nf = buf.shape[1] // W
    out = []
    for i in range(count):
        row = vals[i * nf:(i + 1) * nf]
        d = dict(zip(fields, row[:len(fields)]))
        if nf == 12:
            d["U"] = (row[10], row[11]) if wc else None
        out.append(d)
    return out


def _proof_buf(pfs: Sequence[dict], fields: List[str], nf: int) -> np.ndarray:
    rows = []
    for p in pfs:
        r = [p[f] for f in fields]
        if nf == 12:
            u = p.get("U")
            r += [u[0], u[1]] if u else [0, 0]
        rows.extend(r)
    return np.ascontiguousarray(ints_to_words(rows, W).reshape(len(pfs), nf * W))


def _points(pts: Optional[Sequence[Tuple[int, int]]]) -> Optional[np.ndarray]:
    if pts is None:
        return None
    a = np.zeros((len(pts), 16), dtype="<u4")
    for i, (x, y) in enumerate(pts):
        a[i, :8] = ints_to_words([x], 8)[0]
        a[i, 8:] = ints_to_words([y], 8)[0]
    return a


def _sessions(ss: Sequence[bytes]) -> Tuple[np.ndarray, int]:
    n = len(ss[0]) if ss else 0
    if any(len(s) != n for s in ss):
        raise ValueError("session ids must have equal length")
    return np.frombuffer(b"".join(ss), dtype=np.uint8).copy(), n


def alice_init(pkA_N: int, a: Sequence[int], dlnB: Dict[str, int], seeds: Sequence):
    """AliceInit for a batch -> (cA list, RangeProofAlice list, err list).
    seeds[i]: session i's io.Reader -- an int (CounterDRBG seed) or an object
    with .read(n)."""
    k = _Keep()
    pk, dln = _paillier(k, pkA_N), _dln(k, dlnB)
    n = len(a)
    A = _col(a)
    S = _host.Readers(seeds)
    cA = np.zeros((n, W), dtype="<u4")
    pf = np.zeros((n, 6 * W), dtype="<u4")
    err = np.zeros(n, dtype=np.uint8)
    _check(lib().mpcxh_mta_alice_init_batch(W, ctypes.byref(pk), ctypes.byref(dln), n, A.ctypes.data, S.ptr,
                                            cA.ctypes.data, pf.ctypes.data, err.ctypes.data))
    return words_to_ints(cA), _proofs(pf, RANGE_FIELDS, n), [int(e) for e in err]


def verify_range_alice(pk_N: int, dln_: Dict[str, int], c: Sequence[int], pfs: Sequence[dict]) -> List[bool]:
    k = _Keep()
    pk, dln = _paillier(k, pk_N), _dln(k, dln_)
    n = len(c)
    ok = np.zeros(n, dtype=np.uint8)
    C, P = _col(c), _proof_buf(pfs, RANGE_FIELDS, 6)
    _check(lib().mpcxh_mta_verify_range_alice_batch(W, ctypes.byref(pk), ctypes.byref(dln), n, C.ctypes.data,
                                                    P.ctypes.data, ok.ctypes.data))
    return [bool(x) for x in ok]


def bob_mid(sessions: Sequence[bytes], pkA_N: int, pfA: Sequence[dict], b: Sequence[int], cA: Sequence[int],
            dlnA: Dict[str, int], dlnB: Dict[str, int], seeds: Sequence,
            B: Optional[Sequence[Tuple[int, int]]] = None):
    """BobMid (B None) / BobMidWC -> (beta, cB, betaPrm, ProofBob[WC], err) lists."""
    k = _Keep()
    pk, da, db = _paillier(k, pkA_N), _dln(k, dlnA), _dln(k, dlnB)
    n = len(b)
    ss, sl = _sessions(sessions)
    PA, Bw, CA = _proof_buf(pfA, RANGE_FIELDS, 6), _col(b), _col(cA)
    Bp = _points(B)
    S = _host.Readers(seeds)
    beta, cB, bp = (np.zeros((n, W), dtype="<u4") for _ in range(3))
    pfB = np.zeros((n, 12 * W), dtype="<u4")
    err = np.zeros(n, dtype=np.uint8)
    _check(lib().mpcxh_mta_bob_mid_batch(W, ss.ctypes.data, sl, ctypes.byref(pk), ctypes.byref(da), ctypes.byref(db),
                                         n, PA.ctypes.data, Bw.ctypes.data, CA.ctypes.data, _ptr(Bp), S.ptr,
                                         beta.ctypes.data, cB.ctypes.data, bp.ctypes.data, pfB.ctypes.data,
                                         err.ctypes.data))
    return (words_to_ints(beta), words_to_ints(cB), words_to_ints(bp), _proofs(pfB, BOB_FIELDS, n, B is not None),
            [int(e) for e in err])


def verify_bob(sessions: Sequence[bytes], pk_N: int, dln_: Dict[str, int], c1: Sequence[int], c2: Sequence[int],
               pfs: Sequence[dict], X: Optional[Sequence[Tuple[int, int]]] = None,
               own_sk: Optional[Tuple[int, int, int]] = None) -> List[bool]:
    """(*ProofBob).Verify / (*ProofBobWC).Verify. own_sk = (LambdaN, P, Q) when pk is the caller's."""
    k = _Keep()
    pk = _paillier(k, pk_N, *(own_sk or (None, None, None)))
    dln = _dln(k, dln_)
    n = len(c1)
    ss, sl = _sessions(sessions)
    C1, C2, P = _col(c1), _col(c2), _proof_buf(pfs, BOB_FIELDS, 12)
    Xp = _points(X)
    ok = np.zeros(n, dtype=np.uint8)
    _check(lib().mpcxh_mta_verify_bob_batch(W, ss.ctypes.data, sl, ctypes.byref(pk), ctypes.byref(dln), n,
                                            C1.ctypes.data, C2.ctypes.data, P.ctypes.data, _ptr(Xp), ok.ctypes.data))
    return [bool(x) for x in ok]


def alice_end(sessions: Sequence[bytes], skA: Tuple[int, int, int, int], pfB: Sequence[dict], dlnA: Dict[str, int],
              cA: Sequence[int], cB: Sequence[int], B: Optional[Sequence[Tuple[int, int]]] = None):
    """AliceEnd (B None) / AliceEndWC; skA = (N, LambdaN, P, Q) -> (alpha list, err list)."""
    k = _Keep()
    sk = _paillier(k, *skA)
    dln = _dln(k, dlnA)
    n = len(cA)
    ss, sl = _sessions(sessions)
    P, CA, CB = _proof_buf(pfB, BOB_FIELDS, 12), _col(cA), _col(cB)
    Bp = _points(B)
    alpha = np.zeros((n, W), dtype="<u4")
    err = np.zeros(n, dtype=np.uint8)
    _check(lib().mpcxh_mta_alice_end_batch(W, ss.ctypes.data, sl, ctypes.byref(sk), ctypes.byref(dln), n,
                                           P.ctypes.data, CA.ctypes.data, CB.ctypes.data, _ptr(Bp), alpha.ctypes.data,
                                           err.ctypes.data))
    return words_to_ints(alpha), [int(e) for e in err]


def bob_mid_pair(sessions: Sequence[bytes], pkA_N: int, pfA: Sequence[dict], b: Sequence[int], cA: Sequence[int],
                 dlnA: Dict[str, int], dlnB: Dict[str, int], seeds: Sequence, bwc: Sequence[int],
                 Bwc: Sequence[Tuple[int, int]], seeds_wc: Sequence):
    """BobMid (b, seeds) and BobMidWC (bwc, Bwc, seeds_wc) on the same Alice
    messages in one call -> ((beta, cB, betaPrm, ProofBob, err), (the WC half)).
    seeds_wc is seeds (the same list object): each session's one reader serves
    both halves (the library then runs BobMid before BobMidWC)."""
    k = _Keep()
    pk, da, db = _paillier(k, pkA_N), _dln(k, dlnA), _dln(k, dlnB)
    n = len(b)
    ss, sl = _sessions(sessions)
    PA, Bw, Bwcw, CA = _proof_buf(pfA, RANGE_FIELDS, 6), _col(b), _col(bwc), _col(cA)
    Bp = _points(Bwc)
    S = _host.Readers(seeds)
    Swc = S if seeds_wc is seeds else _host.Readers(seeds_wc)
    outs = []
    for _ in range(2):
        outs.append([np.zeros((n, W), dtype="<u4") for _ in range(3)] + [np.zeros((n, 12 * W), dtype="<u4"),
                                                                         np.zeros(n, dtype=np.uint8)])
    (b1, c1, p1, f1, e1), (b2, c2, p2, f2, e2) = outs
    _check(lib().mpcxh_mta_bob_mid_pair_batch(
        W, ss.ctypes.data, sl, ctypes.byref(pk), ctypes.byref(da), ctypes.byref(db), n, PA.ctypes.data,
        CA.ctypes.data, Bw.ctypes.data, S.ptr, Bwcw.ctypes.data, Bp.ctypes.data, Swc.ptr,
        b1.ctypes.data, c1.ctypes.data, p1.ctypes.data, f1.ctypes.data, e1.ctypes.data,
        b2.ctypes.data, c2.ctypes.data, p2.ctypes.data, f2.ctypes.data, e2.ctypes.data))
    return tuple((words_to_ints(bb), words_to_ints(cc), words_to_ints(pp), _proofs(ff, BOB_FIELDS, n, wc),
                  [int(x) for x in ee]) for (bb, cc, pp, ff, ee), wc in zip(outs, (False, True)))


def alice_end_pair(sessions: Sequence[bytes], skA: Tuple[int, int, int, int], dlnA: Dict[str, int],
                   cA: Sequence[int], pfB: Sequence[dict], cB: Sequence[int], pfB_wc: Sequence[dict],
                   cB_wc: Sequence[int], Bwc: Sequence[Tuple[int, int]]):
    """AliceEnd and AliceEndWC of the same sessions in one call ->
    (alpha list, err list, mu list, err_wc list)."""
    k = _Keep()
    sk = _paillier(k, *skA)
    dln = _dln(k, dlnA)
    n = len(cA)
    ss, sl = _sessions(sessions)
    P1, P2 = _proof_buf(pfB, BOB_FIELDS, 12), _proof_buf(pfB_wc, BOB_FIELDS, 12)
    CA, CB, CBw = _col(cA), _col(cB), _col(cB_wc)
    Bp = _points(Bwc)
    alpha, mu = np.zeros((n, W), dtype="<u4"), np.zeros((n, W), dtype="<u4")
    e1, e2 = np.zeros(n, dtype=np.uint8), np.zeros(n, dtype=np.uint8)
    _check(lib().mpcxh_mta_alice_end_pair_batch(
        W, ss.ctypes.data, sl, ctypes.byref(sk), ctypes.byref(dln), n, CA.ctypes.data, P1.ctypes.data,
        CB.ctypes.data, P2.ctypes.data, CBw.ctypes.data, Bp.ctypes.data, alpha.ctypes.data, e1.ctypes.data,
        mu.ctypes.data, e2.ctypes.data))
    return words_to_ints(alpha), [int(x) for x in e1], words_to_ints(mu), [int(x) for x in e2]


# ---------------------------------------------------------------- test hooks
def sha512_256i(*ints: int, tag: Optional[bytes] = None) -> int:
    n = len(ints)
    A = _col(ints) if n else np.zeros((0, W), dtype="<u4")
    d = (ctypes.c_uint8 * 32)()
    t = (ctypes.c_uint8 * max(1, len(tag or b""))).from_buffer_copy((tag or b"") or b"\0") if tag is not None else None
    _check(lib().mpcxh_sha512_256i(t, len(tag or b""), n, A.ctypes.data, W, d))
    return int.from_bytes(bytes(d), "big")


def _pt_out(a: np.ndarray):
    x, y = words_to_ints(a.reshape(2, 8))
    return None if x == 0 and y == 0 else (x, y)


def scalar_base_mult(k_: int):
    K = _one(k_)
    o = np.zeros(16, dtype="<u4")
    _check(lib().mpcxh_secp_scalar_base_mult(K.ctypes.data, W, o.ctypes.data))
    return _pt_out(o)


def scalar_mult(P: Tuple[int, int], k_: int):
    K = _one(k_)
    Pp = _points([P])
    o = np.zeros(16, dtype="<u4")
    _check(lib().mpcxh_secp_scalar_mult(Pp.ctypes.data, K.ctypes.data, W, o.ctypes.data))
    return _pt_out(o)


def lincomb(u1: int, P: Tuple[int, int], u2: int):
    """u1*G + u2*P on secp256k1 (mpcxh_secp_lincomb)."""
    U1, U2 = _one(u1), _one(u2)
    Pp = _points([P])
    o = np.zeros(16, dtype="<u4")
    _check(lib().mpcxh_secp_lincomb(U1.ctypes.data, Pp.ctypes.data, U2.ctypes.data, W, o.ctypes.data))
    return _pt_out(o)


def random_draws(seed: int, less_than: int, count: int, relprime: bool = False) -> List[int]:
    L = _one(less_than)
    o = np.zeros((count, W), dtype="<u4")
    _check(lib().mpcxh_random_draws(seed, L.ctypes.data, W, 1 if relprime else 0, count, o.ctypes.data))
    return words_to_ints(o)


SIGNING_STATS = ["round1_s", "round2_s", "round3_s", "total_s", "wallets", "sessions", "errors",
                 "relation_failures", "engine_busy_s", "finalize_s", "signatures", "verified", "alg_macs", "aborted"]
TAMPER_R4_SCHNORR, TAMPER_R6_ZKV, TAMPER_R7_DECOMMIT = 1, 2, 3  # signing.hpp kTamper*


def bench_signing(nodes: Sequence[Dict[str, int]], signers: int, wallets: int, seed: int = 0x5167,
                  trace_wallets: int = 0, tamper: Optional[Tuple[int, int]] = None):
    """Config-4 driver (csrc/host/signing.hpp): one GG18 signature for each of
    `wallets` wallets -- MtA / MtAwc on the GPU, rounds 1/4-9 (commitments,
    Schnorr and ZKV proofs, their checks), the signature and ecdsa.Verify.
    nodes: dicts with N, LambdaN, P, Q, NTildei, H1i, H2i, p, q
    (node_preparams.json fields). tamper = (wallet, kind): corrupt that
    wallet's transcript (TAMPER_*; test hook). Returns the stats dict, and with
    trace_wallets > 0 also the trace of the wallets t * wallets // trace_wallets
    (t < trace_wallets; spread over every concurrent wallet pipeline):
    {"wallets": [index], "pairs": [[{alpha, beta, mu, nu, digest} per traced
    wallet] per ordered pair], "sigs": [(r, s, recid)], "gg18": [digest]}."""
    k = _Keep()
    sks = (PaillierKey * len(nodes))(*[_paillier(k, n["N"], n["LambdaN"], n["P"], n["Q"]) for n in nodes])
    dlns = (DLN * len(nodes))(*[_dln(k, {"NTilde": n["NTildei"], "h1": n["H1i"], "h2": n["H2i"],
                                         "P": 2 * n["p"] + 1, "Q": 2 * n["q"] + 1}) for n in nodes])
    st = np.zeros(len(SIGNING_STATS), dtype=np.float64)
    npairs = signers * (signers - 1)
    tw = min(trace_wallets, wallets)
    tr = np.zeros(max(1, npairs * tw * 40 + tw * 25), dtype="<u4")
    tw_idx, tk = tamper if tamper else (-1, 0)
    _check(lib().mpcxh_bench_signing(W, sks, dlns, len(nodes), signers, wallets, seed, st.ctypes.data, tw,
                                     tr.ctypes.data if tw else None, tw_idx, tk))
    stats = dict(zip(SIGNING_STATS, [float(x) for x in st]))
    if not tw:
        return stats
    pairs = []
    for p in range(npairs):
        rows = []
        for wi in range(tw):
            o = (p * tw + wi) * 40
            a, b, m, n_, d = words_to_ints(tr[o:o + 40].reshape(5, 8))
            rows.append({"alpha": a, "beta": b, "mu": m, "nu": n_, "digest": d})
        pairs.append(rows)
    base = npairs * tw * 40
    sigs, gg = [], []
    for wi in range(tw):
        o = base + wi * 25
        r, s = words_to_ints(tr[o:o + 16].reshape(2, 8))
        sigs.append((r, s, int(tr[o + 16])) if r else None)
        gg.append(words_to_ints(tr[o + 17:o + 25].reshape(1, 8))[0] if r else None)
    return stats, {"wallets": [t * wallets // tw for t in range(tw)], "pairs": pairs, "sigs": sigs, "gg18": gg}


def bench_signing_mta(nodes, signers: int, wallets: int, seed: int = 0x5167) -> dict:
    """Back-compatible name of bench_signing (stats only)."""
    return bench_signing(nodes, signers, wallets, seed)
