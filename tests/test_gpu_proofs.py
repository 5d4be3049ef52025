"""GPU parity tests of the batched keygen / reshare proofs (rows A13-A14):
DLN, Paillier-Blum modulus and no-small-factor proofs against the oracle's
golden proofs (tests/golden/proof_vectors.json, oracle/proofs_ref.py), field
by field, plus rejection of tampered proofs with the same decisions as the
oracle."""
import json
import os

import pytest

from conftest import GOLDEN, H
from oracle import proofs_ref as PR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pr(gpu):
    from mpcium_amd import host, proofs
    host.init(0)
    return proofs


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture(scope="module")
def vec():
    return json.load(open(os.path.join(GOLDEN, "proof_vectors.json")))


def test_dln_golden_and_rejections(pr, nodes, vec):
    n0 = nodes[0]
    Nt = n0["NTildei"]
    args = [(n0["H1i"], n0["H2i"], n0["Alpha"]), (n0["H2i"], n0["H1i"], n0["Beta"])]
    for (h1, h2, x), g in zip(args, vec["dln"]):
        got = pr.dln_prove(h1, h2, x, n0["p"], n0["q"], Nt, [g["seed"], g["seed"] + 1000])
        assert got[0]["Alpha"] == [H(v) for v in g["Alpha"]]
        assert got[0]["T"] == [H(v) for v in g["T"]]
        bad_t = {"Alpha": list(got[1]["Alpha"]), "T": list(got[1]["T"])}
        bad_t["T"][5] += 1
        bad_a = {"Alpha": list(got[1]["Alpha"]), "T": list(got[1]["T"])}
        bad_a["Alpha"][127] = 1  # not in (1, N)
        ok = pr.dln_verify(h1, h2, Nt, [got[0], got[1], bad_t, bad_a])
        assert ok == [True, True, False, False]
        assert PR.dln_verify(PR.DLNProof(bad_t["Alpha"], bad_t["T"]), h1, h2, Nt) is False
    # wrong statement: the (h2, h1) proof does not verify for (h1, h2)
    assert pr.dln_verify(n0["H1i"], n0["H2i"], Nt, [got[0]]) == [False]


def test_mod_golden_and_rejections(pr, nodes, vec):
    n0 = nodes[0]
    ss = bytes.fromhex(vec["session"])
    g = vec["mod"]
    got = pr.mod_prove([ss, ss], n0["N"], n0["P"], n0["Q"], [g["seed"], g["seed"] + 1])
    p = got[0]
    assert p["W"] == H(g["W"]) and p["A"] == H(g["A"]) and p["B"] == H(g["B"])
    assert p["X"] == [H(v) for v in g["X"]] and p["Z"] == [H(v) for v in g["Z"]]
    bad_z = dict(got[1], Z=list(got[1]["Z"]))
    bad_z["Z"][3] = (bad_z["Z"][3] + 1) % n0["N"]
    bad_x = dict(got[1], X=list(got[1]["X"]))
    bad_x["X"][79] = (bad_x["X"][79] * 2) % n0["N"]
    bad_a = dict(got[1], A=got[1]["A"] ^ 1)
    other_ss = bytes(32)
    ok = pr.mod_verify([ss, ss, ss, ss, ss, other_ss], n0["N"], [got[0], got[1], bad_z, bad_x, bad_a, got[0]])
    assert ok == [True, True, False, False, False, False]
    # a prime "modulus" is rejected
    P = n0["P"]
    assert pr.mod_verify([ss], P, [got[0]]) == [False]


def test_mod_verify_rejects_prime_modulus_alone(pr, nodes, vec, monkeypatch):
    """ModProof.Verify's N.ProbablyPrime(30) check in isolation: a proof for a
    prime P (a 1024-bit safe prime, P = 3 mod 4) that satisfies every equation
    -- the oracle accepts it once its primality check is disabled -- is rejected
    by the GPU verifier and the oracle. A composite N with its honest proof in
    the same batch verifies."""
    from oracle import safeprime_ref as SP
    from oracle import tss_ref as T
    n0 = nodes[0]
    ss = bytes.fromhex(vec["session"])
    P = n0["P"]
    crafted = PR.mod_proof_for_prime(ss, P, T.Reader(0x9F1E))
    assert PR.mod_verify(crafted, ss, P) is False
    monkeypatch.setattr(SP, "probably_prime", lambda n, reps=20: False)
    assert PR.mod_verify(crafted, ss, P) is True  # every other check passes
    monkeypatch.undo()
    honest = pr.mod_prove([ss], n0["N"], n0["P"], n0["Q"], [vec["mod"]["seed"]])[0]
    pf = {"W": crafted.W, "X": list(crafted.X), "A": crafted.A, "B": crafted.B, "Z": list(crafted.Z)}
    assert pr.mod_verify([ss], P, [pf]) == [False]
    assert pr.mod_verify([ss], n0["N"], [honest]) == [True]


def test_fac_golden_and_rejections(pr, nodes, vec):
    n0, n1 = nodes[0], nodes[1]
    ss = bytes.fromhex(vec["session"])
    g = vec["fac"]
    args = (n0["N"], n1["NTildei"], n1["H1i"], n1["H2i"])
    got = pr.fac_prove([ss, ss], *args, n0["P"], n0["Q"], [g["seed"], g["seed"] + 1])
    assert {k: got[0][k] for k in pr.FAC_FIELDS} == {k: H(g[k]) for k in pr.FAC_FIELDS}
    cases = [got[0], got[1]]
    for f in ("Z1", "W2", "V", "Sigma", "T"):
        c = dict(got[1])
        c[f] += 1
        cases.append(c)
    neg = dict(got[1])
    neg["V"] = -neg["V"]  # exercises the negative-exponent path (must fail)
    cases.append(neg)
    # z1 / z2 shifted by the order of the QR subgroup mod N~: the equations
    # hold, only the z range check rejects (tests/test_proofs_cpu.py)
    order = n1["p"] * n1["q"]
    for dz1, dz2 in ((order, 0), (0, order), (2 * order, order)):
        c = dict(got[0])
        c["Z1"] += dz1
        c["Z2"] += dz2
        cases.append(c)
    ok = pr.fac_verify([ss] * len(cases), *args, cases)
    assert ok == [True, True] + [False] * (len(cases) - 2)
    for c, o in zip(cases, ok):
        assert PR.fac_verify(PR.FacProof(**c), ss, *args) == o
    # FacVerify folds R^e into s^(N0 e) t^(Sigma e), so a peer's Sigma
    # sets the length of a per-operand exponent. Over-long Sigma (off the group
    # order, and shifted by a multiple of it, which leaves R unchanged), V = -1,
    # and an honest proof in the same batch: the same decisions as the oracle,
    # and nothing else in the batch fails (a field wider than the C-ABI's W words
    # is rejected by the wrapper, proofs.fac_verify)
    odd = []
    for dsig in (1 << 6000, order << 3000, -1):
        c = dict(got[0])
        c["Sigma"] += dsig
        odd.append(c)
    c = dict(got[0])
    c["V"] = -1
    odd += [c, got[0]]
    ok2 = pr.fac_verify([ss] * len(odd), *args, odd)
    want = [PR.fac_verify(PR.FacProof(**c), ss, *args) for c in odd]
    assert ok2 == want
    assert ok2[0] is False and ok2[-1] is True
    # the proof is bound to the verifier's N~
    n2 = nodes[2]
    assert pr.fac_verify([ss], n0["N"], n2["NTildei"], n2["H1i"], n2["H2i"], [got[0]]) == [False]


def test_keygen_proof_driver_small():
    """Config-5 driver (csrc/host/keygenload.hpp) on the 3 fixture nodes:
    every party's DLN x2 / Mod / Fac proofs verify at every peer."""
    import json
    import os
    from mpcium_amd import host as mhost
    from mpcium_amd import proofs as mproofs
    mhost.init(0)
    with open(os.path.join(os.path.dirname(__file__), "golden", "node_preparams.json")) as f:
        nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"}
                 for n in json.load(f)["nodes"]]
    st = mproofs.bench_keygen_proofs(nodes, 3, seed=5)
    assert st["failures"] == 0
    assert st["proofs"] == 3 * 3 * (3 + 2) and st["verifications"] == 3 * 3 * 2 * 4
