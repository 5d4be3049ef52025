#!/usr/bin/env python3
"""Generate tests/golden/proof_vectors.json: keygen proofs (SURVEY.md 8(a)
A13-A14) computed by oracle/proofs_ref.py over CounterDRBG readers on the
nodes of node_preparams.json:
  dln: node 0's two round-1 proofs (h1, h2, alpha) and (h2, h1, beta) over N~_0
  mod: node 0's Paillier-Blum proof of N_0 (session id below)
  fac: node 0's no-small-factor proof of N_0 over node 1's (N~, h1, h2)
Each proof is asserted to verify here; the GPU path must reproduce every field."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import proofs_ref as PR  # noqa: E402
from oracle import tss_ref as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "proof_vectors.json")
SEED = 0x70726630  # "prf0"


def h(v):
    return ("-" + format(-v, "x")) if v < 0 else format(v, "x")


def main():
    t0 = time.time()
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "node_preparams.json")))
    nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"}
             for n in d["nodes"]]
    n0, n1 = nodes[0], nodes[1]
    session = T.Reader(SEED).read(32)
    dln1 = PR.dln_prove(n0["H1i"], n0["H2i"], n0["Alpha"], n0["p"], n0["q"], n0["NTildei"], T.Reader(SEED + 1))
    dln2 = PR.dln_prove(n0["H2i"], n0["H1i"], n0["Beta"], n0["p"], n0["q"], n0["NTildei"], T.Reader(SEED + 2))
    assert PR.dln_verify(dln1, n0["H1i"], n0["H2i"], n0["NTildei"])
    assert PR.dln_verify(dln2, n0["H2i"], n0["H1i"], n0["NTildei"])
    mod = PR.mod_prove(session, n0["N"], n0["P"], n0["Q"], T.Reader(SEED + 3))
    assert PR.mod_verify(mod, session, n0["N"])
    fac = PR.fac_prove(session, n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"], n0["P"], n0["Q"], T.Reader(SEED + 4))
    assert PR.fac_verify(fac, session, n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"])
    out = {
        "description": "keygen proofs from oracle/proofs_ref.py (tests/golden/gen_proofs.py); node 0 proves, "
                       "fac over node 1's N~",
        "session": session.hex(),
        "dln": [{"seed": SEED + 1, "Alpha": [h(v) for v in dln1.Alpha], "T": [h(v) for v in dln1.T]},
                {"seed": SEED + 2, "Alpha": [h(v) for v in dln2.Alpha], "T": [h(v) for v in dln2.T]}],
        "mod": {"seed": SEED + 3, "W": h(mod.W), "X": [h(v) for v in mod.X], "A": h(mod.A), "B": h(mod.B),
                "Z": [h(v) for v in mod.Z]},
        "fac": {"seed": SEED + 4, **{k: h(getattr(fac, k)) for k in
                                     ("P", "Q", "A", "B", "T", "Sigma", "Z1", "Z2", "W1", "W2", "V")}},
    }
    out["gen_seconds"] = round(time.time() - t0, 1)
    json.dump(out, open(OUT, "w"), indent=1)
    print("wrote", OUT, out["gen_seconds"], "s")


if __name__ == "__main__":
    main()
