"""GPU tests of BASELINE configs 4 and 5 through the C-ABI drivers.

Config 4 (csrc/host/signing.hpp, mpcxh_bench_signing): 1,000 wallets signed by
2 and by 3 of the 3 fixture nodes (3 = every ready peer, mpcium's default:
/root/reference/pkg/mpc/node.go:148). The driver checks alpha + beta = k gamma
and mu + nu = k w on every session and ecdsa.Verify on every signature; sampled
wallets are recomputed by the oracle (oracle/signing_ref.py) and compared field
by field: every pair's alpha, beta, mu, nu, a digest of the whole session
transcript (cA, both proofs, cB, cB'), a digest of the GG18 round 1/4-9
transcript (commitments, Schnorr and ZKV proofs, s_i) and the signature
(r, s, recid). A tampered proof or decommitment aborts its wallet only.

Config 5 (csrc/host/keygenload.hpp): 5-party keygen / reshare proof work
(3-of-5), streamed in waves, every proof verified, one session per wave
compared with the oracle (oracle/keygen_ref.py)."""
import json
import os

import pytest

from conftest import GOLDEN
from oracle import crosscheck as cc
from oracle import mta_ref as M
from oracle import signing_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture(scope="module")
def drv(gpu):
    from mpcium_amd import host, mta
    host.init(0)
    return mta


@pytest.fixture()
def fast_exp():
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    old = M._pw
    M._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    yield
    M._pw = old


@pytest.mark.parametrize("signers,wallets,trace", [(2, 10000, 6), (3, 10000, 6)])
def test_signing_wallets_match_oracle(drv, nodes, fast_exp, signers, wallets, trace):
    """Config 4 at its stated size, 10,000 wallets, for 2 signers (three
    concurrent wallet pipelines by default) and 3 signers (mpcium's default,
    every ready peer; two pipelines): traced wallets are spread over the batch,
    so every pipeline's sessions are compared with the oracle."""
    seed = 0x516E + signers
    st, tr = drv.bench_signing(nodes, signers, wallets, seed=seed, trace_wallets=trace)
    assert st["errors"] == 0 and st["relation_failures"] == 0
    assert st["signatures"] == wallets and st["verified"] == wallets
    assert st["sessions"] == wallets * signers * (signers - 1)
    order = S.pair_order(signers)
    assert tr["wallets"] == [t * wallets // trace for t in range(trace)]
    if signers == 2:  # one traced wallet in each third (the default pipelines' chunks)
        assert {wi * 3 // wallets for wi in tr["wallets"]} == {0, 1, 2}
    else:  # and in each half
        assert {wi * 2 // wallets for wi in tr["wallets"]} == {0, 1}
    assert st["aborted"] == 0
    for t, wi in enumerate(tr["wallets"]):
        pairs, sig, ok, gg18 = S.sign_wallet(nodes, signers, seed, wi)
        assert ok
        assert tr["sigs"][t] == sig, wi
        assert tr["gg18"][t] == gg18, wi  # rounds 1, 4-9: commitments, Schnorr / ZKV proofs, s_i
        for p, ij in enumerate(order):
            assert tr["pairs"][p][t] == pairs[ij], (wi, ij)


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_tampered_transcript_aborts_only_its_wallet(drv, nodes, fast_exp, kind):
    """A corrupted round-4 Schnorr proof, round-6 ZKV proof or round-7
    decommitment of one signer in one wallet aborts that wallet only (the
    oracle aborts it too); every other wallet is signed and verified, and a
    traced honest wallet still matches the oracle."""
    seed, wallets, bad = 0x7A3F, 96, 37
    st, tr = drv.bench_signing(nodes, 2, wallets, seed=seed, trace_wallets=2, tamper=(bad, kind))
    assert st["errors"] == 0 and st["relation_failures"] == 0
    assert st["aborted"] == 1 and st["signatures"] == wallets - 1 and st["verified"] == wallets - 1
    _, sig, ok, _ = S.sign_wallet(nodes, 2, seed, bad, tamper=kind)
    assert sig is None and not ok
    pairs, sig, ok, gg18 = S.sign_wallet(nodes, 2, seed, tr["wallets"][1])
    assert ok and tr["sigs"][1] == sig and tr["gg18"][1] == gg18


@pytest.fixture(scope="module")
def five_parties(drv, nodes):
    """The 3 fixture nodes plus 2 nodes whose preparams come from the GPU
    GeneratePreParams (config 5 is 3-of-5)."""
    from mpcium_amd import host as mhost
    parties = list(nodes)
    for seed in (0x6D706335, 0x6D706336):
        pp, _ = mhost.generate_preparams(seed=seed)
        assert pp["N"] == pp["P"] * pp["Q"] and pp["NTildei"] == (2 * pp["p"] + 1) * (2 * pp["q"] + 1)
        parties.append(pp)
    return parties


def test_keygen_reshare_waves_match_oracle(five_parties):
    """Config 5's driver streaming sessions in bounded-memory waves (3 waves of
    32 sessions here): every party proves DLN x2, Mod and a Fac proof per peer
    and verifies every peer's proofs; one traced session per wave is recomputed
    by the oracle (oracle/keygen_ref.py) and every proof's digest compared, and
    the wave split changes no proof (same traced session, other wave size)."""
    from mpcium_amd import proofs as mproofs
    from oracle import keygen_ref as KR
    from oracle import proofs_ref as PR
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    n, sessions, wave, seed = 5, 96, 32, 0x6B69
    st, tr = mproofs.bench_keygen_proofs(five_parties, sessions, seed=seed, wave=wave, trace=True)
    assert st["failures"] == 0
    assert st["waves"] == 3 and st["wave_sessions"] == wave
    assert st["proofs"] == sessions * n * (2 + 1 + (n - 1))
    assert st["verifications"] == sessions * n * (n - 1) * 4
    assert [t["session"] for t in tr] == [w * wave + (w * 7919) % wave for w in range(3)]
    old = PR._pw
    PR._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    try:
        for t in tr:
            want, passed = KR.session_digests(five_parties, seed, t["session"])
            assert t["digests"] == want, t["session"]
            assert t["verified"] == passed == n * (n - 1) * 4
    finally:
        PR._pw = old
    # the same sessions in one wave of 96: the traced session 0's proofs are unchanged
    st1, tr1 = mproofs.bench_keygen_proofs(five_parties, sessions, seed=seed, wave=sessions, trace=True)
    assert st1["failures"] == 0 and st1["waves"] == 1
    assert tr1[0]["session"] == tr[0]["session"] == 0
    assert tr1[0]["digests"] == tr[0]["digests"]


def test_keygen_bench_wave_size_matches_oracle(five_parties):
    """Config 5 at the bench's wave size: one wave of 1,024 concurrent
    sessions (bench.py keygen_line's default), every proof of every session
    verified by every peer, and the wave's traced session recomputed by the
    oracle proof by proof."""
    from mpcium_amd import proofs as mproofs
    from oracle import keygen_ref as KR
    from oracle import proofs_ref as PR
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    n, sessions, seed = 5, 1024, 0x6B6A
    st, tr = mproofs.bench_keygen_proofs(five_parties, sessions, seed=seed, wave=sessions, trace=True)
    assert st["failures"] == 0
    assert st["waves"] == 1 and st["wave_sessions"] == sessions
    assert st["verifications"] == sessions * n * (n - 1) * 4
    (t,) = tr
    old = PR._pw
    PR._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    try:
        want, passed = KR.session_digests(five_parties, seed, t["session"])
    finally:
        PR._pw = old
    assert t["digests"] == want, t["session"]
    assert t["verified"] == passed == n * (n - 1) * 4


def test_keygen_reshare_mix_matches_oracle(five_parties):
    """Config 5 with resharing as mpcium runs it (an old-party and a new-party
    session per node per wallet): odd waves are resharing waves -- the new
    committee's proofs plus the old committee's VSS (commitments and shares on
    the GPU EC kernel) and the new committee's decommitment, share and
    public-key checks. One traced session per wave vs the oracle: every proof
    digest, and on resharing waves the VSS digests, the new shares and the
    count of passed checks (oracle/keygen_ref.py reshare_vss)."""
    from mpcium_amd import proofs as mproofs
    from oracle import keygen_ref as KR
    from oracle import proofs_ref as PR
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    n, sessions, wave, seed = 5, 128, 32, 0x6B6B
    st, tr = mproofs.bench_keygen_proofs(five_parties, sessions, seed=seed, wave=wave, trace=True, reshare=True)
    assert st["failures"] == 0 and st["vss_failures"] == 0
    assert st["keygen_sessions"] == st["reshare_sessions"] == sessions // 2
    assert st["vss_checks"] == st["reshare_sessions"] * (n * n + n)
    old = PR._pw
    PR._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    try:
        for w, t in enumerate(tr):
            want, passed = KR.session_digests(five_parties, seed, t["session"])
            assert t["digests"] == want, t["session"]
            assert t["verified"] == passed == n * (n - 1) * 4
            if w % 2 == 1:
                digs, shares, good = KR.reshare_vss(n, seed, t["session"])
                assert t["vss"] == {"old": digs, "new_shares": shares, "passed": good}
                assert good == n * n + n
            else:
                assert "vss" not in t
    finally:
        PR._pw = old


def test_reshare_tampered_share_fails_only_its_check(five_parties):
    """A resharing session where old party 0 sends new party 1 a share off by
    one: exactly that one VSS check fails (s_01 G != sum_k V_0k 2^k), every
    other check of every session and every proof still passes, and the traced
    session of that wave reports one check fewer."""
    from mpcium_amd import proofs as mproofs
    n, sessions, wave, seed = 5, 64, 32, 0x6B6C
    tr_session = 32 + (1 * 7919) % 32  # wave 1 (a resharing wave): its traced session
    st, tr = mproofs.bench_keygen_proofs(five_parties, sessions, seed=seed, wave=wave, trace=True, reshare=True,
                                         tamper_session=tr_session)
    assert st["failures"] == 0
    assert st["vss_failures"] == 1
    assert st["vss_checks"] == st["reshare_sessions"] * (n * n + n)
    assert tr[1]["session"] == tr_session and tr[1]["vss"]["passed"] == n * n + n - 1
