"""CPU tests of the keygen-proof oracle (rows A13-A14): the restatement
reproduces and verifies its golden proofs, rejects tampered ones, and its
Jacobi symbol agrees with Euler's criterion."""
import json
import os

import pytest

from conftest import GOLDEN, H
from oracle import proofs_ref as PR
from oracle import tss_ref as T


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture(scope="module")
def vec():
    return json.load(open(os.path.join(GOLDEN, "proof_vectors.json")))


def test_jacobi_matches_euler():
    for p in (3, 5, 7, 11, 13, 10007, 2 ** 127 - 1):
        for a in list(range(0, 40)) + [p - 1, p + 5, 3 * p]:
            e = pow(a, (p - 1) // 2, p)
            assert PR.jacobi(a, p) == (0 if a % p == 0 else (1 if e == 1 else -1))
    assert PR.jacobi(2, 15) == 1 and PR.jacobi(7, 15) == -1 and PR.jacobi(5, 15) == 0


def test_fac_oracle_reproduces_golden(nodes, vec):
    n0, n1 = nodes[0], nodes[1]
    ss = bytes.fromhex(vec["session"])
    g = vec["fac"]
    pf = PR.fac_prove(ss, n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"], n0["P"], n0["Q"], T.Reader(g["seed"]))
    assert {k: getattr(pf, k) for k in ("P", "Q", "A", "B", "T", "Sigma", "Z1", "Z2", "W1", "W2", "V")} == \
        {k: H(g[k]) for k in ("P", "Q", "A", "B", "T", "Sigma", "Z1", "Z2", "W1", "W2", "V")}
    assert PR.fac_verify(pf, ss, n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"])
    pf.Z2 += 1
    assert not PR.fac_verify(pf, ss, n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"])


def fac_equations_hold(pf, ss, N0, NCap, s, t):
    """The three verification equations of (*ProofFac).Verify, without the
    range checks."""
    e = T.rejection_sample(PR.Q, T.sha512_256i_tagged(ss, N0, NCap, s, t, pf.P, pf.Q, pf.A, pf.B, pf.T, pf.Sigma))
    M = NCap
    tv = pow(t, pf.V, M) if pf.V >= 0 else pow(pow(t, -1, M), -pf.V, M)
    R = pow(s, N0, M) * pow(t, pf.Sigma, M) % M
    return (pow(s, pf.Z1, M) * pow(t, pf.W1, M) % M == pf.A * pow(pf.P, e, M) % M and
            pow(s, pf.Z2, M) * pow(t, pf.W2, M) % M == pf.B * pow(pf.Q, e, M) % M and
            pow(pf.Q, pf.Z1, M) * tv % M == pf.T * pow(R, e, M) % M)


def shifted_fac_proofs(pf, nodes):
    """z1 or z2 moved by the order p'q' of the quadratic residues mod N~ =
    (2p'+1)(2q'+1), where s, t, P, Q, A, B, T all live: every equation still
    holds, and only the z range check can reject the proof (the
    bound that makes the no-small-factor proof sound)."""
    import dataclasses
    order = nodes[1]["p"] * nodes[1]["q"]
    return [dataclasses.replace(pf, Z1=pf.Z1 + order), dataclasses.replace(pf, Z2=pf.Z2 + order),
            dataclasses.replace(pf, Z1=pf.Z1 + 2 * order, Z2=pf.Z2 + order)]


def test_fac_z_range_rejects_shifted_responses(nodes, vec):
    n0, n1 = nodes[0], nodes[1]
    ss = bytes.fromhex(vec["session"])
    g = vec["fac"]
    args = (n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"])
    pf = PR.fac_prove(ss, *args[:4], n0["P"], n0["Q"], T.Reader(g["seed"]))
    assert fac_equations_hold(pf, ss, *args) and PR.fac_verify(pf, ss, *args)
    import math
    bound = (PR.Q ** 3 + 2 * PR.Q) * math.isqrt(n0["N"])
    assert pf.Z1 <= bound and pf.Z2 <= bound
    for bad in shifted_fac_proofs(pf, nodes):
        assert fac_equations_hold(bad, ss, *args)
        assert not PR.fac_verify(bad, ss, *args)


def test_mod_and_dln_golden_verify(nodes, vec):
    n0 = nodes[0]
    ss = bytes.fromhex(vec["session"])
    g = vec["mod"]
    pf = PR.ModProof(H(g["W"]), [H(v) for v in g["X"]], H(g["A"]), H(g["B"]), [H(v) for v in g["Z"]])
    assert PR.mod_verify(pf, ss, n0["N"])
    pf.B ^= 2
    assert not PR.mod_verify(pf, ss, n0["N"])
    d = vec["dln"][0]
    dp = PR.DLNProof([H(v) for v in d["Alpha"]], [H(v) for v in d["T"]])
    assert PR.dln_verify(dp, n0["H1i"], n0["H2i"], n0["NTildei"])
