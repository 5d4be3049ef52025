"""GPU parity tests of the batched MtA / MtAwc mirror (rows A8-A10) against
the oracle's golden sessions (tests/golden/mta_vectors.json, made by
oracle/mta_ref.py): every output field bit-exact, error codes for tampered
proofs and bad inputs, and the MtA relations on a larger random batch."""
import json
import os

import pytest

from conftest import GOLDEN, H
from oracle import mta_ref as M
from oracle import tss_ref as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mta(gpu):
    from mpcium_amd import host, mta
    host.init(0)
    return mta


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture(scope="module")
def vec():
    return json.load(open(os.path.join(GOLDEN, "mta_vectors.json")))["sessions"]


def dln(n, own=False):
    d = {"NTilde": n["NTildei"], "h1": n["H1i"], "h2": n["H2i"]}
    if own:
        d["P"], d["Q"] = 2 * n["p"] + 1, 2 * n["q"] + 1
    return d


def hx(d):
    return {k: (H(v) if isinstance(v, str) else v) for k, v in d.items()}


def bob_pf(d, wc):
    p = {k: H(d[k]) for k in M.ProofBob.__dataclass_fields__ if k != "U"}
    p["U"] = (H(d["Ux"]), H(d["Uy"])) if wc else None
    return p


def by_pair(vec):
    """Golden sessions grouped by (Alice node, Bob node): one batch per pair."""
    out = {}
    for v in vec:
        out.setdefault((v["alice_node"], v["bob_node"]), []).append(v)
    return out


@pytest.mark.parametrize("pair", [(0, 1), (1, 0), (1, 2), (2, 1), (2, 0), (0, 2)])
def test_golden_sessions_bit_exact(mta, nodes, vec, pair):
    """39 golden sessions over all 6 ordered node pairs, every field bit-exact."""
    vec = by_pair(vec)[pair]
    A, B = nodes[pair[0]], nodes[pair[1]]
    n = len(vec)
    a = [H(v["a"]) for v in vec]
    cA, pfA, err = mta.alice_init(A["N"], a, dln(B), [v["seed_a"] for v in vec])
    assert err == [0] * n
    assert cA == [H(v["cA"]) for v in vec]
    assert pfA == [hx(v["pfA"]) for v in vec]
    ss = [bytes.fromhex(v["session"]) for v in vec]
    Bpts = [(H(v["Bx"]), H(v["By"])) for v in vec]
    for wc, key, bs, seeds in ((False, "bob", [H(v["b"]) for v in vec], [v["seed_b"] for v in vec]),
                               (True, "bob_wc", [H(v["wB"]) for v in vec], [v["seed_bwc"] for v in vec])):
        beta, cB, bp, pfB, err = mta.bob_mid(ss, A["N"], pfA, bs, cA, dln(A), dln(B, own=True), seeds,
                                             B=Bpts if wc else None)
        assert err == [0] * n, key
        assert beta == [H(v[key]["beta"]) for v in vec], key
        assert cB == [H(v[key]["cB"]) for v in vec], key
        assert bp == [H(v[key]["betaPrm"]) for v in vec], key
        assert pfB == [bob_pf(v[key]["pf"], wc) for v in vec], key
        sk = (A["N"], A["LambdaN"], A["P"], A["Q"])
        alpha, err = mta.alice_end(ss, sk, pfB, dln(A, own=True), cA, cB, B=Bpts if wc else None)
        assert err == [0] * n, key
        assert alpha == [H(v["alpha_wc" if wc else "alpha"]) for v in vec], key


@pytest.mark.parametrize("pair", [(0, 1), (2, 0)])
def test_golden_sessions_paired_entries(mta, nodes, vec, pair):
    """BobMid + BobMidWC and AliceEnd + AliceEndWC as one paired call each
    (signing rounds 2 and 3): every field equals the golden sessions; a tampered
    range proof fails both halves, a tampered ProofBobWC only its own half."""
    vec = by_pair(vec)[pair]
    A, B = nodes[pair[0]], nodes[pair[1]]
    n = len(vec)
    ss = [bytes.fromhex(v["session"]) for v in vec]
    Bpts = [(H(v["Bx"]), H(v["By"])) for v in vec]
    pfA = [hx(v["pfA"]) for v in vec]
    bad = dict(pfA[0])
    bad["S2"] += 1
    pfA_in = [bad] + pfA[1:]
    cA = [H(v["cA"]) for v in vec]
    plain, wc = mta.bob_mid_pair(ss, A["N"], pfA_in, [H(v["b"]) for v in vec], cA, dln(A), dln(B, own=True),
                                 [v["seed_b"] for v in vec], [H(v["wB"]) for v in vec], Bpts,
                                 [v["seed_bwc"] for v in vec])
    for (beta, cB, bp, pfB, err), key, is_wc in ((plain, "bob", False), (wc, "bob_wc", True)):
        assert err == [mta.ERR_PROOF_VERIFY] + [0] * (n - 1), key
        assert beta[1:] == [H(v[key]["beta"]) for v in vec[1:]], key
        assert cB[1:] == [H(v[key]["cB"]) for v in vec[1:]], key
        assert bp[1:] == [H(v[key]["betaPrm"]) for v in vec[1:]], key
        assert pfB[1:] == [bob_pf(v[key]["pf"], is_wc) for v in vec[1:]], key
    sk = (A["N"], A["LambdaN"], A["P"], A["Q"])
    pf1 = [bob_pf(v["bob"]["pf"], False) for v in vec]
    pf2 = [bob_pf(v["bob_wc"]["pf"], True) for v in vec]
    pf2[-1] = dict(pf2[-1], T2=pf2[-1]["T2"] + 1)
    alpha, e1, mu, e2 = mta.alice_end_pair(ss, sk, dln(A, own=True), cA, pf1, [H(v["bob"]["cB"]) for v in vec], pf2,
                                           [H(v["bob_wc"]["cB"]) for v in vec], Bpts)
    assert e1 == [0] * n and e2 == [0] * (n - 1) + [mta.ERR_PROOF_VERIFY]
    assert alpha == [H(v["alpha"]) for v in vec]
    assert mu[:-1] == [H(v["alpha_wc"]) for v in vec[:-1]]


def test_range_proof_rejections(mta, nodes, vec):
    A, B = nodes[0], nodes[1]
    v = vec[0]
    c, pf = H(v["cA"]), hx(v["pfA"])
    bad = []
    for f, delta in (("S1", 1), ("S2", 1), ("Z", 1), ("U", 1), ("W", 1), ("S", 1)):
        p = dict(pf)
        p[f] += delta
        bad.append(p)
    p = dict(pf)
    p["S1"] = M.Q ** 3 + 1  # out of range
    bad.append(p)
    p = dict(pf)
    p["Z"] = B["NTildei"]  # not in [0, N~)
    bad.append(p)
    p = dict(pf)
    p["S"] = A["P"]  # gcd(S, N) != 1
    bad.append(p)
    cs = [c] * (len(bad) + 2) + [c + 1]
    pfs = [pf] + bad + [pf, pf]
    ok = mta.verify_range_alice(A["N"], dln(B), cs, pfs)
    assert ok == [True] + [False] * len(bad) + [True, False]
    # same decisions as the oracle
    for cc, p, o in zip(cs, pfs, ok):
        assert M.verify_range_alice(M.RangeProofAlice(**p), A["N"], B["NTildei"], B["H1i"], B["H2i"], cc) == o


def test_bob_mid_rejects_bad_range_proof_and_b(mta, nodes, vec):
    A, B = nodes[0], nodes[1]
    v = vec[0]
    pf = hx(v["pfA"])
    bad = dict(pf)
    bad["S"] = (bad["S"] + 1) % A["N"]
    ss = [bytes.fromhex(v["session"])] * 3
    beta, cB, bp, pfB, err = mta.bob_mid(ss, A["N"], [pf, bad, pf], [H(v["b"]), H(v["b"]), A["N"]],
                                         [H(v["cA"])] * 3, dln(A), dln(B), [v["seed_b"]] * 3)
    assert err == [0, mta.ERR_PROOF_VERIFY, mta.ERR_MESSAGE_TOO_LONG]
    assert cB[0] == H(v["bob"]["cB"]) and beta[0] == H(v["bob"]["beta"])


def test_bob_proof_rejections(mta, nodes, vec):
    A = nodes[0]
    v = vec[0]
    ss = bytes.fromhex(v["session"])
    c1, c2 = H(v["cA"]), H(v["bob_wc"]["cB"])
    X = (H(v["Bx"]), H(v["By"]))
    pf = bob_pf(v["bob_wc"]["pf"], True)
    cases = [(pf, ss, X, True)]
    for f in ("Z", "ZPrm", "T", "V", "W", "S", "S1", "S2", "T1", "T2"):
        p = dict(pf)
        p[f] += 1
        cases.append((p, ss, X, False))
    p = dict(pf)
    p["U"] = T.ec_add(pf["U"], T.SECP_G)
    cases.append((p, ss, X, False))                       # wrong u
    cases.append((pf, ss[:-1] + bytes([ss[-1] ^ 1]), X, False))  # other session
    cases.append((pf, ss, T.ec_add(X, T.SECP_G), False))  # other X
    p = dict(pf)
    p["S1"] = M.Q ** 3 + 1
    cases.append((p, ss, X, False))
    p = dict(pf)
    p["T1"] = M.Q ** 7 + 1                                 # t1 above the q^7 bound
    cases.append((p, ss, X, False))
    sk = (A["LambdaN"], A["P"], A["Q"])
    for own in (None, sk):
        ok = mta.verify_bob([c[1] for c in cases], A["N"], dln(A, own=own is not None), [c1] * len(cases),
                            [c2] * len(cases), [c[0] for c in cases], X=[c[2] for c in cases], own_sk=own)
        assert ok == [c[3] for c in cases]
    # plain ProofBob: verify the non-WC golden proof, WC-only fields ignored
    pfp = bob_pf(v["bob"]["pf"], False)
    assert mta.verify_bob([ss], A["N"], dln(A), [c1], [H(v["bob"]["cB"])], [pfp]) == [True]


def test_random_batch_relations(mta, nodes):
    """64 sessions per direction for every ordered node pair, with the MtA
    relations alpha + beta = a*b (mod q) checked on every session."""
    q = M.Q
    rd = T.Reader(0xBA7C4)
    for ia, ib in ((0, 1), (1, 2), (2, 0)):
        A, B = nodes[ia], nodes[ib]
        n = 64
        a = [T.get_random_positive_int(rd, q) for _ in range(n)]
        b = [T.get_random_positive_int(rd, q) for _ in range(n)]
        ss = [rd.read(32) for _ in range(n)]
        seeds = [1000 * ia + 10 * ib + i for i in range(n)]
        cA, pfA, err = mta.alice_init(A["N"], a, dln(B), seeds)
        assert err == [0] * n
        Bp = [T.scalar_base_mult(x) for x in b]
        beta, cB, _, pfB, err = mta.bob_mid(ss, A["N"], pfA, b, cA, dln(A), dln(B, own=True),
                                            [s + 7 for s in seeds], B=Bp)
        assert err == [0] * n
        alpha, err = mta.alice_end(ss, (A["N"], A["LambdaN"], A["P"], A["Q"]), pfB, dln(A, own=True), cA, cB, B=Bp)
        assert err == [0] * n
        assert [(x + y) % q for x, y in zip(alpha, beta)] == [x * y % q for x, y in zip(a, b)]


@pytest.mark.parametrize("pair", [(0, 1), (2, 0)])
def test_golden_sessions_through_reader_callbacks(mta, nodes, vec, pair):
    """The same golden sessions with every random draw made through the
    io.Reader callback (mpcxh_reader_t.fn -> a Python reader object called from
    libmpcx_host's worker threads), as a Go integration threads tss-lib's
    party reader through the batch entry points."""
    vec = by_pair(vec)[pair]
    A, B = nodes[pair[0]], nodes[pair[1]]
    n = len(vec)
    a = [H(v["a"]) for v in vec]
    cA, pfA, err = mta.alice_init(A["N"], a, dln(B), [T.Reader(v["seed_a"]) for v in vec])
    assert err == [0] * n
    assert cA == [H(v["cA"]) for v in vec]
    assert pfA == [hx(v["pfA"]) for v in vec]
    ss = [bytes.fromhex(v["session"]) for v in vec]
    Bpts = [(H(v["Bx"]), H(v["By"])) for v in vec]
    beta, cB, bp, pfB, err = mta.bob_mid(ss, A["N"], pfA, [H(v["wB"]) for v in vec], cA, dln(A), dln(B, own=True),
                                         [T.Reader(v["seed_bwc"]) for v in vec], B=Bpts)
    assert err == [0] * n
    assert cB == [H(v["bob_wc"]["cB"]) for v in vec]
    assert pfB == [bob_pf(v["bob_wc"]["pf"], True) for v in vec]


def test_overlong_exponent_does_not_fail_the_batch(mta, nodes, vec, monkeypatch):
    """a peer-supplied exponent far above any protocol bound (a
    70,000-bit S2 in one of 80 range proofs) takes the per-operand path; the
    honest proofs of the same batch still verify and the bad one is
    rejected -- one adversarial input never throws for the whole batch."""
    A, B = nodes[0], nodes[1]
    v = vec[0]
    c, pf = H(v["cA"]), hx(v["pfA"])
    bad = dict(pf)
    bad["S2"] = (1 << 70000) + 12345
    monkeypatch.setattr(mta, "W", 2240)  # integer width (words) that carries a 70,000-bit field
    pfs = [pf] * 79 + [bad]
    ok = mta.verify_range_alice(A["N"], dln(B), [c] * 80, pfs)
    assert ok == [True] * 79 + [False]


def test_bob_mid_rejects_ciphertext_above_n2(mta, nodes, vec, monkeypatch):
    """a range proof made for cA + N^2 verifies (Verify reduces c,
    the hash binds it as given), but HomoMult(b, cA) requires cA < N^2: BobMid
    must return ErrMessageTooLong, as Go and the oracle do; the honest session
    beside it is unaffected."""
    A, B = nodes[0], nodes[1]
    v = vec[0]
    N2 = A["N"] ** 2
    rd = T.Reader(v["seed_a"])
    cA, rA = M.encrypt_and_return_randomness(rd, A["N"], H(v["a"]))
    assert cA == H(v["cA"])
    big = cA + N2
    pf_big = M.prove_range_alice(A["N"], big, B["NTildei"], B["H1i"], B["H2i"], H(v["a"]), rA, rd)
    assert M.verify_range_alice(pf_big, A["N"], B["NTildei"], B["H1i"], B["H2i"], big)
    with pytest.raises(M.ErrMessageTooLong):
        M.bob_mid(bytes.fromhex(v["session"]), A["N"], pf_big, H(v["b"]), big, A["NTildei"], A["H1i"], A["H2i"],
                  B["NTildei"], B["H1i"], B["H2i"], T.Reader(v["seed_b"]))
    monkeypatch.setattr(mta, "W", 160)  # cA + N^2 has 4097 bits
    pf_big = {f: getattr(pf_big, f) for f in M.RangeProofAlice.__dataclass_fields__}
    ss = [bytes.fromhex(v["session"])] * 2
    beta, cB, bp, pfB, err = mta.bob_mid(ss, A["N"], [hx(v["pfA"]), pf_big], [H(v["b"])] * 2, [cA, big], dln(A),
                                         dln(B), [v["seed_b"]] * 2)
    assert err == [0, mta.ERR_MESSAGE_TOO_LONG]
    assert cB[0] == H(v["bob"]["cB"])


def test_bob_mid_pair_with_one_reader_per_session(mta, nodes, vec):
    """one callback reader object passed for both halves of each
    session (as a tss-lib integration passing the party's reader to BobMid and
    BobMidWC) is never called concurrently: the pair entry then equals BobMid
    followed by BobMidWC on the same readers."""
    vec = by_pair(vec)[(0, 1)]
    A, B = nodes[0], nodes[1]
    n = len(vec)
    ss = [bytes.fromhex(v["session"]) for v in vec]
    Bpts = [(H(v["Bx"]), H(v["By"])) for v in vec]
    pfA, cA = [hx(v["pfA"]) for v in vec], [H(v["cA"]) for v in vec]
    bs, ws = [H(v["b"]) for v in vec], [H(v["wB"]) for v in vec]
    shared = [T.Reader(0x5EED + i) for i in range(n)]
    plain, wc = mta.bob_mid_pair(ss, A["N"], pfA, bs, cA, dln(A), dln(B, own=True), shared, ws, Bpts, shared)
    sep = [T.Reader(0x5EED + i) for i in range(n)]
    want_plain = mta.bob_mid(ss, A["N"], pfA, bs, cA, dln(A), dln(B, own=True), sep)
    want_wc = mta.bob_mid(ss, A["N"], pfA, ws, cA, dln(A), dln(B, own=True), sep, B=Bpts)
    assert plain == want_plain
    assert wc == want_wc
    assert plain[4] == [0] * n and wc[4] == [0] * n
