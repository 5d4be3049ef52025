#!/usr/bin/env python3
"""Generate tests/golden/mta_vectors.json: MtA / MtAwc sessions computed by the
Python restatement (oracle/mta_ref.py) over the CounterDRBG readers, on the
nodes of node_preparams.json.  Sessions 0-2 run Alice = node 0 (Paillier
key), Bob = node 1; sessions 3-38 run 6 sessions on each of the 6 ordered node
pairs (fields "alice_node" / "bob_node").

Per session: AliceInit (Alice's reader seed_a) -> BobMid and BobMidWC (Bob's
readers seed_b, seed_bwc; B = w*G) -> AliceEnd and AliceEndWC. Every output is
recorded (cA, both proofs, beta, cB, betaPrm, alpha) so the GPU path can be
compared field by field; the MtA relations alpha + beta = a*b (mod q) are
asserted here.
"""
from __future__ import annotations

import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import mta_ref as M  # noqa: E402
from oracle import tss_ref as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "mta_vectors.json")
SEED = 0x6D746130  # "mta0"


def h(v):
    return format(v, "x")


def load_nodes():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"}
            for n in d["nodes"]]


PAIRS = [(0, 1)] * 3 + [p for p in ((0, 1), (1, 0), (1, 2), (2, 1), (2, 0), (0, 2)) for _ in range(6)]


def session(args):
    s, ia, ib, a, b, wB, ssid = args
    nodes = load_nodes()
    A, B = nodes[ia], nodes[ib]
    q = M.Q
    seed_a, seed_b, seed_bwc = SEED + 16 * s + 1, SEED + 16 * s + 2, SEED + 16 * s + 3
    Bpt = T.scalar_base_mult(wB)
    cA, pfA = M.alice_init(A["N"], a, B["NTildei"], B["H1i"], B["H2i"], T.Reader(seed_a))
    beta, cB, beta_prm, piB = M.bob_mid(ssid, A["N"], pfA, b, cA, A["NTildei"], A["H1i"], A["H2i"],
                                        B["NTildei"], B["H1i"], B["H2i"], T.Reader(seed_b))
    beta_wc, cB_wc, beta_prm_wc, piB_wc = M.bob_mid(ssid, A["N"], pfA, wB, cA, A["NTildei"], A["H1i"],
                                                    A["H2i"], B["NTildei"], B["H1i"], B["H2i"],
                                                    T.Reader(seed_bwc), B=Bpt, wc=True)
    alpha = M.alice_end(ssid, A["N"], piB, A["H1i"], A["H2i"], cA, cB, A["NTildei"], A["LambdaN"])
    alpha_wc = M.alice_end(ssid, A["N"], piB_wc, A["H1i"], A["H2i"], cA, cB_wc, A["NTildei"], A["LambdaN"],
                           B=Bpt, wc=True)
    assert (alpha + beta) % q == a * b % q
    assert (alpha_wc + beta_wc) % q == a * wB % q

    def bob(p):
        d = {k: h(getattr(p, k)) for k in ("Z", "ZPrm", "T", "V", "W", "S", "S1", "S2", "T1", "T2")}
        if p.U is not None:
            d["Ux"], d["Uy"] = h(p.U[0]), h(p.U[1])
        return d

    return {
        "alice_node": ia, "bob_node": ib,
        "a": h(a), "b": h(b), "wB": h(wB), "session": ssid.hex(), "Bx": h(Bpt[0]), "By": h(Bpt[1]),
        "seed_a": seed_a, "seed_b": seed_b, "seed_bwc": seed_bwc,
        "cA": h(cA), "pfA": {k: h(getattr(pfA, k)) for k in ("Z", "U", "W", "S", "S1", "S2")},
        "bob": {"beta": h(beta), "cB": h(cB), "betaPrm": h(beta_prm), "pf": bob(piB)},
        "bob_wc": {"beta": h(beta_wc), "cB": h(cB_wc), "betaPrm": h(beta_prm_wc), "pf": bob(piB_wc)},
        "alpha": h(alpha), "alpha_wc": h(alpha_wc),
    }


def main():
    t0 = time.time()
    q = M.Q
    seeds_rd = T.Reader(SEED)
    jobs = []
    for s, (ia, ib) in enumerate(PAIRS):
        a = T.get_random_positive_int(seeds_rd, q)
        b = T.get_random_positive_int(seeds_rd, q)
        wB = T.get_random_positive_int(seeds_rd, q)
        jobs.append((s, ia, ib, a, b, wB, seeds_rd.read(32)))
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        sessions = pool.map(session, jobs, chunksize=1)
    json.dump({"description": "MtA/MtAwc sessions from oracle/mta_ref.py (tests/golden/gen_mta.py) on the nodes "
                              "of node_preparams.json; each session names its Alice and Bob node",
               "seed": SEED, "gen_seconds": round(time.time() - t0, 1), "sessions": sessions},
              open(OUT, "w"), indent=1)
    print("wrote", OUT, round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
