#!/usr/bin/env python3
"""Generate tests/golden/node_preparams.json: three synthetic mpcium nodes'
keygen.LocalPreParams (up:ecdsa/keygen/prepare.go; restated in SURVEY.md 8(a)
A7, A11), used by the MtA parity tests and the signing benchmark (config 4).

Node 0's Paillier key is the existing paillier_key_2048.json key. Every other
prime is the first safe prime of the tss-lib candidate stream
(oracle/safeprime_ref.py) over the CounterDRBG seeded as recorded; Paillier
keys retry the second prime until |P - Q| has >= 1021 bits. N~ = P'Q' with
P' = 2p+1, Q' = 2q+1; f, alpha uniform in Z*_N~ (GetRandomPositiveRelativelyPrimeInt
over the CounterDRBG), h1 = f^2, h2 = h1^alpha mod N~, beta = alpha^-1 mod pq.

Pure Python (pow); the 12 safe-prime searches run in parallel processes
(~1-3 min on 8 cores).
"""
from __future__ import annotations

import json
import math
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import safeprime_ref as sp  # noqa: E402
from oracle import tss_ref as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "node_preparams.json")
SEED_BASE = 0x6D706E00  # "mpn\0"


def h(v: int) -> str:
    return format(v, "x")


def first_safe_prime(seed: int):
    idx, p, q = sp.first_safe_primes(seed, 1024, 1)[0]
    return seed, idx, p, q


def main():
    t0 = time.time()
    key0 = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))
    # seeds: node n uses SEED_BASE + 64 n + {0..}: Paillier P, Q (Q retried upward), N~ p', q'
    jobs = {}
    for n in range(3):
        b = SEED_BASE + 64 * n
        if n > 0:
            jobs[(n, "P")] = b
            for k in range(4):  # Q candidates (first one with |P-Q| large enough wins)
                jobs[(n, f"Q{k}")] = b + 1 + k
        jobs[(n, "Pt")] = b + 16
        jobs[(n, "Qt")] = b + 17
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        res = dict(zip(jobs.keys(), ex.map(first_safe_prime, jobs.values())))
    nodes = []
    for n in range(3):
        if n == 0:
            P, Q = int(key0["P"], 16), int(key0["Q"], 16)
            pk_src = "paillier_key_2048.json"
        else:
            P = res[(n, "P")][2]
            Q = None
            for k in range(4):
                cand = res[(n, f"Q{k}")][2]
                if abs(P - cand).bit_length() >= 1024 - 3 and cand != P:
                    Q, pk_src = cand, f"seeds P={res[(n, 'P')][0]:#x} Q={res[(n, f'Q{k}')][0]:#x}"
                    break
            assert Q is not None
        N = P * Q
        phi = (P - 1) * (Q - 1)
        lam = phi // math.gcd(P - 1, Q - 1)
        _, _, Pt, pt = res[(n, "Pt")]
        _, _, Qt, qt = res[(n, "Qt")]
        Nt = Pt * Qt
        rd = T.Reader(SEED_BASE + 64 * n + 32)
        f = T.get_random_positive_relatively_prime_int(rd, Nt)
        alpha = T.get_random_positive_relatively_prime_int(rd, Nt)
        pq = pt * qt
        beta = pow(alpha, -1, pq)
        h1 = f * f % Nt
        h2 = pow(h1, alpha, Nt)
        nodes.append({
            "paillier_source": pk_src,
            "N": h(N), "P": h(P), "Q": h(Q), "LambdaN": h(lam), "PhiN": h(phi),
            "NTildei": h(Nt), "H1i": h(h1), "H2i": h(h2), "Alpha": h(alpha), "Beta": h(beta),
            "p": h(pt), "q": h(qt),
            "seeds": {"Pt": res[(n, "Pt")][0], "Qt": res[(n, "Qt")][0], "f_alpha_reader": SEED_BASE + 64 * n + 32},
        })
    json.dump({"description": "Three synthetic nodes' LocalPreParams (tests/golden/gen_nodes.py)",
               "gen_seconds": round(time.time() - t0, 1), "nodes": nodes}, open(OUT, "w"), indent=1)
    print("wrote", OUT, round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
