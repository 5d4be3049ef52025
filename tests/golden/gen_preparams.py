#!/usr/bin/env python3
"""Generate tests/golden/preparams_vectors.json with the oracle (test
infrastructure, run offline; the GPU path must reproduce every field):

* safe_primes_1024: the first two 1024-bit safe primes of the CounterDRBG(15)
  candidate stream (tss-lib runGenPrimeRoutine at concurrency 1,
  oracle/safeprime_ref.py), with their stream indices;
* preparams: keygen.GeneratePreParams on the CounterDRBG(0x70726570) stream
  (oracle/safeprime_ref.py generate_preparams: Paillier search, then N~'s,
  then f and alpha, each search consuming the stream exactly through its last
  accepted candidate) -- all 12 LocalPreParams fields and the bytes consumed.

The candidate tests run on a process pool in stream-order chunks (the first
accepted candidate of a chunk is the same as in a one-by-one walk); the
chunked walk is checked against oracle.safeprime_ref.first_safe_primes on a
512-bit stream before use.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import safeprime_ref as S  # noqa: E402
from oracle import tss_ref as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "preparams_vectors.json")
CHUNK = 2048


class OffsetDRBG:
    """CounterDRBG bytes by absolute offset (same stream as oracle/gomath.py)."""

    def __init__(self, seed: int):
        self.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.pos = 0

    def block(self, c: int) -> bytes:
        return hashlib.sha256(b"mpcx-drbg" + self.seed.to_bytes(8, "little") + c.to_bytes(8, "little")).digest()

    def at(self, off: int, n: int) -> bytes:
        out = b"".join(self.block(c) for c in range(off // 32, (off + n + 31) // 32))
        s = off % 32
        return out[s:s + n]

    def read(self, n: int) -> bytes:
        b = self.at(self.pos, n)
        self.pos += n
        return b


def _check(args):
    q, qb = args
    return S.is_safe_prime_pair(q, qb)


def search(rng: OffsetDRBG, p_bits: int, num: int, pool):
    """First num safe primes from rng's position; rng left right after the last one."""
    qb = p_bits - 1
    nb = (qb + 7) // 8
    out, idx0 = [], 0
    while True:
        start = rng.pos
        raw = rng.at(start, CHUNK * nb)
        qs = [S.candidate_from_bytes(raw[i * nb:(i + 1) * nb], qb) for i in range(CHUNK)]
        flags = pool.map(_check, [(q, qb) for q in qs], chunksize=32)
        for i, ok in enumerate(flags):
            if ok:
                out.append((idx0 + i, 2 * qs[i] + 1, qs[i]))
                if len(out) == num:
                    rng.pos = start + (i + 1) * nb
                    return out
        rng.pos = start + CHUNK * nb
        idx0 += CHUNK


def preparams(seed: int, pool):
    rng = OffsetDRBG(seed)
    while True:
        sg = search(rng, 1024, 2, pool)
        P, Q = sg[0][1], sg[1][1]
        if abs(P - Q).bit_length() >= 1024 - 3:
            break
    phi = (P - 1) * (Q - 1)
    lam = phi // math.gcd(P - 1, Q - 1)
    sg = search(rng, 1024, 2, pool)
    Pt, Qt, p, q = sg[0][1], sg[1][1], sg[0][2], sg[1][2]
    NT = Pt * Qt
    f1 = T.get_random_positive_relatively_prime_int(rng, NT)
    alpha = T.get_random_positive_relatively_prime_int(rng, NT)
    h1 = f1 * f1 % NT
    return {"N": P * Q, "LambdaN": lam, "PhiN": phi, "P": P, "Q": Q, "NTildei": NT, "H1i": h1,
            "H2i": pow(h1, alpha, NT), "Alpha": alpha, "Beta": pow(alpha, -1, p * q), "p": p, "q": q,
            "consumed_bytes": rng.pos}


def main():
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        # the chunked parallel walk equals the oracle's one-by-one walk
        ref = S.first_safe_primes(21, 512, 2)
        got = search(OffsetDRBG(21), 512, 2, pool)
        assert [(i, p) for i, p, _ in ref] == [(i, p) for i, p, _ in got], (ref, got)
        sp = search(OffsetDRBG(15), 1024, 2, pool)
        pp = preparams(0x70726570, pool)
    h = lambda v: format(v, "x")  # noqa: E731
    doc = {"description": "oracle/safeprime_ref.py restatement (tests/golden/gen_preparams.py): first 1024-bit "
                          "safe primes of a CounterDRBG candidate stream, and GeneratePreParams on one stream",
           "safe_primes_1024": {"seed": 15, "primes": [{"index": i, "p": h(p), "q": h(q)} for i, p, q in sp]},
           "preparams": {"seed": 0x70726570, **{k: (h(v) if k != "consumed_bytes" else v) for k, v in pp.items()}},
           "gen_seconds": round(time.time() - t0, 1)}
    json.dump(doc, open(OUT, "w"), indent=1)
    print("wrote", OUT, round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
